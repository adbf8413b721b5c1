# Round 6: C3 pipeline with the pre-round-6 wave kernel vs the in-place LDS layout (same box)
set -u
A="--config C3 --no-cpu-baseline --no-serialized"
OUT=${OUT:-r6f} BENCH_LIMIT=200 RUNS="c3new:$A|c3old@ASR_LIB=libasr_amd_cv_oldwave.so:$A|c3new4:$A --inflight 4 --prod-streams 4|c3new5:$A --inflight 5 --prod-streams 5|c3old5@ASR_LIB=libasr_amd_cv_oldwave.so:$A --inflight 5 --prod-streams 5|c3newb:$A|c3oldb@ASR_LIB=libasr_amd_cv_oldwave.so:$A" bash tools/bench_matrix.sh
