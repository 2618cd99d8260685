import os, sys, torch, torch.nn.functional as F
sys.path.insert(0, os.getcwd())
from grace_amd.models import resnet50, resnet18
DEV = "cuda"
for name, fn, b, r in (("resnet18", resnet18, 8, 64), ("resnet50", resnet50, 4, 64), ("resnet50", resnet50, 16, 112)):
    torch.manual_seed(0)
    model = fn().to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(b, 3, r, r, device=DEV).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (b,), device=DEV)
    out = {}
    for tag, force in (("f1", "0"), ("u1", "1"), ("f2", "0"), ("u2", "1")):
        os.environ["GRACE_AMD_FORCE_TORCH"] = force
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), y)
        loss.backward()
        out[tag] = (loss.item(), [p.grad.float().reshape(-1).clone() for p in model.parameters()])
    os.environ["GRACE_AMD_FORCE_TORCH"] = "0"
    names = [n for n, _ in model.named_parameters()]
    def cos(a, b, idx=None):
        A = torch.cat(out[a][1] if idx is None else [out[a][1][i] for i in idx]); B = torch.cat(out[b][1] if idx is None else [out[b][1][i] for i in idx])
        return F.cosine_similarity(A, B, dim=0).item()
    print(name, b, r, "loss", {k: round(v[0], 5) for k, v in out.items()})
    print("  all  f1-u1 %.4f  u1-u2 %.4f  f1-f2 %.4f" % (cos("f1", "u1"), cos("u1", "u2"), cos("f1", "f2")))
    for i in (0, 1, 2, len(names) - 5, len(names) - 3, len(names) - 2, len(names) - 1):
        print("  %-28s f1-u1 %.4f u1-u2 %.4f f1-f2 %.4f  |f| %.3e |u| %.3e" % (names[i], cos("f1", "u1", [i]), cos("u1", "u2", [i]), cos("f1", "f2", [i]), out["f1"][1][i].norm().item(), out["u1"][1][i].norm().item()))
