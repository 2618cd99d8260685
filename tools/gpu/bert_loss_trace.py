"""BERT-base (BASELINE config 5) loss per step: eager torch.optim.SGD vs eager FusedSGD vs the
whole-step HIP graph with FusedSGD, 30 steps each from the same initial weights (VERDICT r4 item 2:
bench.py's bert rows ended at NaN).  The eager runs also name the first parameter whose
gradient goes non-finite.  Usage: python tools/gpu/bert_loss_trace.py [--workload bert_none]
"""
import argparse
import copy
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from grace_amd import grace_from_params  # noqa: E402
from grace_amd.parallel import DistributedOptimizer, FusedSGD  # noqa: E402
from grace_amd.parallel.graph import GraphedStep  # noqa: E402
from grace_amd.utils.workloads import WORKLOADS, build_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="bert_none")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--modes", default="eager_torch,eager_fused,graph_fused")
    ap.add_argument("--dropout", type=float, default=None, help="override the model's dropout")
    ap.add_argument("--benchmark", action="store_true", help="torch.backends.cudnn.benchmark = True (as bench.py)")
    ap.add_argument("--cap-warm", type=int, default=3)
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = args.benchmark
    dev = torch.device("cuda", 0)
    torch.backends.cuda.matmul.allow_tf32 = False
    w = WORKLOADS[args.workload]
    torch.manual_seed(0)
    base = build_model(w, dev)
    if args.dropout is not None:
        for m in base.modules():
            if hasattr(m, "p") and isinstance(m.p, float):
                m.p = args.dropout
    init = copy.deepcopy(base.state_dict())
    data = w.make_batch(w.batch, dev)
    for mode in args.modes.split(","):
        torch.manual_seed(1)
        model = base
        model.load_state_dict(init)
        named = list(model.named_parameters())
        params = [p for _, p in named]
        base_opt = torch.optim.SGD(params, lr=0.01, momentum=0.5) if mode == "eager_torch" \
            else FusedSGD(params, lr=0.01, momentum=0.5)
        grc = grace_from_params(dict(w.grace, world_size=1))
        opt = DistributedOptimizer(base_opt, grc, named_parameters=named, bucket_cap_mb=128.0, overlap=False)
        first_bad = None

        def step():
            opt.zero_grad(set_to_none=True)
            loss = w.loss(model, data)
            loss.backward()
            opt.step()
            return loss

        losses = []
        if mode.startswith("graph"):
            run = GraphedStep(step, warmup=args.cap_warm)
            for _ in range(args.steps - args.cap_warm):
                losses.append(float(run().item()))
        else:
            for i in range(args.steps):
                opt.zero_grad(set_to_none=True)
                loss = w.loss(model, data)
                loss.backward()
                if first_bad is None:
                    for n, p in named:
                        if p.grad is not None and not torch.isfinite(p.grad).all():
                            first_bad = (i, n)
                            break
                opt.step()
                losses.append(float(loss.item()))
        if mode.startswith("graph"):
            # eager steps continuing from the graphed run's weights: does the state stay sane?
            for _ in range(3):
                opt.zero_grad(set_to_none=True)
                loss = w.loss(model, data)
                loss.backward()
                opt.step()
                losses.append(float(loss.item()))
        wmax = max(float(p.detach().abs().max()) for p in params)
        print(json.dumps({"workload": args.workload, "mode": mode, "dropout": args.dropout, "losses": [round(v, 4) for v in losses],
                          "first_nonfinite_grad": first_bad, "max_abs_weight": wmax}), flush=True)
        opt.engine.remove()


if __name__ == "__main__":
    main()
