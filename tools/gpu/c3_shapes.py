"""Every conv3x3 backend vs MIOpen on the resnet18_cifar (batch 8, 16x16) conv shapes."""
import torch
from grace_amd.ops import conv as CV

torch.manual_seed(0)
shapes = [(8, 16, 16, 64, 64, 1, 3), (8, 16, 16, 64, 128, 2, 3), (8, 8, 8, 128, 128, 1, 3), (8, 8, 8, 128, 256, 2, 3),
          (8, 4, 4, 256, 256, 1, 3), (8, 4, 4, 256, 512, 2, 3), (8, 2, 2, 512, 512, 1, 3),
          (8, 16, 16, 64, 128, 2, 1), (8, 8, 8, 128, 256, 2, 1), (8, 4, 4, 256, 512, 2, 1)]
cl = torch.channels_last
for nb, h, wd, cin, cout, s, k in shapes:
    x = torch.randn(nb, cin, h, wd, device="cuda").contiguous(memory_format=cl)
    w = (torch.randn(cout, cin, k, k, device="cuda") * 0.05).contiguous(memory_format=cl)
    ho = (h - 1) // s + 1
    dy = torch.randn(nb, cout, ho, ho, device="cuda").contiguous(memory_format=cl)
    for d in ("fwd", "dgrad", "wgrad"):
        ref = CV._run3(d, "miopen", x, w, dy, s).float()
        for be in CV.C3_BACKENDS[1:]:
            try:
                got = CV._run3(d, be, x, w, dy, s)
            except Exception as e:
                continue
            torch.cuda.synchronize()
            err = float((got - ref).abs().max()) / (float(ref.abs().max()) + 1e-12)
            flag = "  <-- BAD" if err > 1e-4 else ""
            if flag:
                print(f"{(nb, h, wd, cin, cout, s, k)} {d} {be} rel err {err:.2e}{flag}", flush=True)
print("done", flush=True)
