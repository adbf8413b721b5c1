# The round-5 bench scan summary (profiles/r05/bench_scan.md) from gpurun_out/.
python tools/bench_scan.py profiles/r05/bench_scan.md \
  "sa:first line with stages / clock / placement fields (before the round-5 decoder changes)" \
  "sb:short fp64 lse + emission prefetch by 32-bit offsets; production GEMM order A/B (knob removed)" \
  "sc:emission prefetch through per-chunk buffer resources (VGPR spills gone), full line with parity" \
  "sd:decode partition 128 / 144 / 160 at 256 and 512 per GPU; shard sizes" \
  "se:fragment-major P (ASR_PIPELINE_PFRAG on / off)" \
  "sf:256 per GPU: decodes in flight, production streams, segments, GEMM tiles per workgroup (t4 / t16); C2 on CU groups" \
  "sg:C2: CU groups vs the chip-filling schedule (D 6 / 10 / 12, one segment, 60 steps)" \
  "sh:C2 chip-filling variants (192 decode CUs, 16-22 decodes, 32 queues); C4 at 32 queues" \
  "si:full default lines (CPU baseline, parity witness): C4 and C2" \
  "sj:shards 1024 / 512 / 256, C3, C5, BL" \
  "sk:C4 decode partition 112-136; C5 decode slicing / decodes in flight" \
  "sl:production over every CU while the pipeline fills (ASR_PIPELINE_FILL, removed); at 24 queues only 512 and C4 took it" \
  "sm:fill at 32 queues (256 per GPU); whole-XCD CU masks (ASR_PIPELINE_XCD, removed)" \
  "sn:GPU_MAX_HW_QUEUES 4 / 8 / 16 / 24 / 32 (queue fit: production streams first)" \
  "sn2:4 / 8 / 16 queues, queue fit: the larger of D / P first" \
  "so:4 / 8 / 16 queues, queue fit: production streams down to half the decodes, then both (the product)" \
  "c5n:C5 and BL after the wide decoder's superset-test candidates (13.2 us per frame)" \
  "c5s:C5 T-segments 2 / 3 / 4 (13.2 us decoder)" \
  "fin_r5c:final tree (12.3 us wide decoder): C4, C2 with parity witness; C5, BL" \
  "$@"
