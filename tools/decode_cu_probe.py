"""Decode kernel time vs utterances per CU on a CU-masked stream (the
pipeline's decode partition): is the one-wave decoder one round at 16 per
CU, and how does a batch's time grow past a round?

    python tools/decode_cu_probe.py [--T 300] [--cus 128] [--per-cu 8,15,16,17,24,32]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
import bench  # noqa: E402
from __graft_entry__ import PKG, _load  # noqa: E402

asr = _load("asr_amd", PKG / "asr_amd.py")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=300)
    ap.add_argument("--cus", type=int, default=128)
    ap.add_argument("--per-cu", default="8,15,16,17,24,32")
    ap.add_argument("--beam", type=int, default=50)
    ap.add_argument("--V", type=int, default=29)
    args = ap.parse_args()
    import torch
    asr.set_device(0)
    torch.cuda.set_device(0)
    from ctc_profile import bench_emissions
    ks = [int(x) for x in args.per_cu.split(",")]
    Bmax = max(ks) * args.cus
    emis = bench_emissions(args.T, Bmax, args.V)
    d_em = asr.DeviceMatrix.from_numpy(emis.reshape(args.T * Bmax, args.V))
    st = bench.cu_range_stream(0, args.cus)
    for k in ks:
        B = k * args.cus
        dec = asr.CTCDecoder(args.V, args.beam, 0, waves=asr.ASR_CTC_WAVES_LIST)
        ms = []
        for _ in range(3):
            dec.decode_device(d_em.ptr, args.T, B, True, stream=st.cuda_stream, frame_stride=Bmax * args.V,
                              utt_stride=args.V)
            dec.best()
            ms.append(dec.last_kernel_ms())
        dec.close()
        t = min(ms)
        print(json.dumps({"cus": args.cus, "per_cu": k, "B": B, "T": args.T, "kernel_ms": round(t, 4),
                          "us_per_frame": round(1e3 * t / args.T, 3),
                          "utt_frames_per_us_per_cu": round(B * args.T / (t * 1e3) / args.cus, 4)}), flush=True)
    bench.destroy_raw_streams()


if __name__ == "__main__":
    main()
