"""Per-layer A/B of the ResNet-50 b32 fp32 3x3 convolutions: MIOpen (its zero fills included) vs
the implicit GEMM on the f32 MFMA kernel (gemm_f32.hip modes 2-4), per direction and tile."""
import torch

from grace_amd.ops import conv as CV

LAYERS = [  # (N, Cin, H, W, Cout, stride, count in ResNet-50)
    (32, 64, 56, 56, 64, 1, 3), (32, 128, 56, 56, 128, 2, 1), (32, 128, 28, 28, 128, 1, 3),
    (32, 256, 28, 28, 256, 2, 1), (32, 256, 14, 14, 256, 1, 5), (32, 512, 14, 14, 512, 2, 1),
    (32, 512, 7, 7, 512, 1, 2),
    # the strided 1x1 projection shortcuts (ksize 1, pad 0)
    (32, 256, 56, 56, 512, 2, -1), (32, 512, 28, 28, 1024, 2, -1), (32, 1024, 14, 14, 2048, 2, -1)]
tot = {"miopen": 0.0, "best": 0.0}
print(f"{'layer':34s} {'dir':6s} " + " ".join(f"{b:>8s}" for b in CV.C3_BACKENDS) + "   TF/s(best)")
for N, Cin, H, W, Cout, s, cnt in LAYERS:
    ks = 1 if cnt < 0 else 3
    cnt = abs(cnt)
    x = torch.randn(N, Cin, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, ks, ks, device="cuda") * 0.05).contiguous(memory_format=torch.channels_last)
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    dy = torch.randn(N, Cout, Ho, Wo, device="cuda").contiguous(memory_format=torch.channels_last)
    flops = 2.0 * N * Ho * Wo * Cout * Cin * ks * ks
    for d in ("fwd", "dgrad", "wgrad"):
        row = {}
        for be in CV.C3_BACKENDS:
            try:
                row[be] = CV._time(lambda: CV._run3(d, be, x, w, dy, s), reps=20)
            except Exception:
                row[be] = float("nan")
        ok = {k: v for k, v in row.items() if v == v}
        best = min(ok, key=ok.get)
        tot["miopen"] += cnt * row["miopen"]
        tot["best"] += cnt * ok[best]
        print(f"{str((N, Cin, H, W, Cout, s, ks)):34s} {d:6s} " + " ".join(f"{row[b]:8.4f}" for b in CV.C3_BACKENDS)
              + f"   {flops / ok[best] / 1e9:6.1f} {best}", flush=True)
print(f"network 3x3 total (ms per step, x multiplicity): miopen {tot['miopen']:.3f}  best {tot['best']:.3f}")
