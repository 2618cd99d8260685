"""BERT whole-step graph replayed back to back (no host sync between replays, as bench.py's timed
loop), every replay's loss copied on the device and printed at the end.  Variants switch off the
attention-probability dropout (inside scaled_dot_product_attention) or the hidden-state dropouts
(F.dropout) separately, to find which random op goes wrong under unsynchronised replays.
Usage: python tools/gpu/bert_graph_nosync.py --variant {both,attn_only,hidden_only,none} [--sync]
"""
import argparse
import os
import sys
import types

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from grace_amd import grace_from_params  # noqa: E402
from grace_amd.models import bert as bert_mod  # noqa: E402
from grace_amd.parallel import DistributedOptimizer, FusedSGD  # noqa: E402
from grace_amd.parallel.graph import GraphedStep  # noqa: E402
from grace_amd.utils.workloads import WORKLOADS, build_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="both")
    ap.add_argument("--replays", type=int, default=40)
    ap.add_argument("--sync", action="store_true")
    ap.add_argument("--sync-at", type=int, default=-1, help="one device sync after this replay only")
    ap.add_argument("--sdpa-math", action="store_true", help="force the math SDPA backend")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    attn = args.variant in ("both", "attn_only")
    hidden = args.variant in ("both", "hidden_only")
    ns = types.SimpleNamespace(**{k: getattr(F, k) for k in dir(F) if not k.startswith("__")})
    if not attn:
        ns.scaled_dot_product_attention = lambda q, k, v, attn_mask=None, dropout_p=0.0: \
            F.scaled_dot_product_attention(q, k, v, attn_mask=attn_mask, dropout_p=0.0)
    if not hidden:
        ns.dropout = lambda x, p=0.5, training=True, inplace=False: x
    bert_mod.F = ns
    w = WORKLOADS["bert_none"]
    torch.manual_seed(0)
    model = build_model(w, dev)
    named = list(model.named_parameters())
    opt = DistributedOptimizer(FusedSGD([p for _, p in named], lr=0.01, momentum=0.5),
                               grace_from_params(dict(w.grace, world_size=1)), named_parameters=named,
                               bucket_cap_mb=128.0, overlap=False)
    data = w.make_batch(w.batch, dev)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = w.loss(model, data)
        loss.backward()
        opt.step()
        return loss

    import contextlib

    ctx = contextlib.nullcontext()
    if args.sdpa_math:
        from torch.nn.attention import SDPBackend, sdpa_kernel

        ctx = sdpa_kernel([SDPBackend.MATH])
    with ctx:
        run = GraphedStep(step, warmup=5)
        rec = torch.empty(args.replays, device=dev)
        for i in range(args.replays):
            loss = run()
            rec[i].copy_(loss.float().reshape(()))
            if args.sync or i == args.sync_at:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
    vals = rec.tolist()
    first_bad = next((i for i in range(1, len(vals)) if not (vals[i] == vals[i]) or vals[i] > vals[i - 1] + 0.5), None)
    print(f"variant={args.variant} sync={args.sync} sync_at={args.sync_at} math={args.sdpa_math} first_jump={first_bad} "
          + " ".join(f"{v:.3f}" for v in vals), flush=True)


if __name__ == "__main__":
    main()
