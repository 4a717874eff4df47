"""Calibration: the vendor GEMM (torch.mm -> hipBLASLt/rocBLAS) on the search shapes, output
materialised (unlike the fused kernel). Gives the practical MFMA ceiling of this K = 768 shape.
Usage: python tools/gemm_calibrate.py"""
import json

import torch


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    out = []
    for n, b, dt in ((90000, 1024, torch.bfloat16), (90000, 4096, torch.bfloat16), (5_000_000, 1024, torch.float16)):
        c = torch.randn(n, 768, device=dev, dtype=dt)
        q = torch.randn(768, b, device=dev, dtype=dt)
        for _ in range(3):
            torch.mm(c, q)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20 if n < 1_000_000 else 3
        e0.record()
        for _ in range(reps):
            s = torch.mm(c, q)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        fl = 2.0 * n * b * 768
        out.append({"rows": n, "batch": b, "dtype": str(dt), "ms": round(ms, 4), "TFLOPs": round(fl / ms / 1e9, 1),
                    "out_bytes": s.numel() * s.element_size()})
        del c, q, s
    print(json.dumps(out))


if __name__ == "__main__":
    main()
