#!/usr/bin/env python3
"""grace_amd benchmark: data-parallel training throughput with GRACE gradient compression.

Headline (BASELINE.json): ResNet-50, ImageNet shape 3x224x224, batch 32 per GPU, Top-K 1% +
ResidualMemory + Allgather, SGD(lr = 0.01 * W, momentum 0.5) -- the reference harness
/root/reference/examples/torch/pytorch_synthetic_benchmark.py:46-55, 110-111, 151-154 with
``Allgather(TopKCompressor(0.01), ResidualMemory())`` (line 119).  Synthetic data and
random-init weights (no datasets / checkpoints offline).

    python bench.py --gpus 1 --steps 20 --warmup 10
    python bench.py --gpus 8 --steps 20 --warmup 10          # launches its own 8 ranks
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 10

``--gpus N > 1`` without torchrun's ``WORLD_SIZE``: the script re-launches itself as N ranks
through grace_amd/launcher.py (the ``horovodrun -np N`` role, /root/reference/TRAINING.md:69-73):
fresh child processes started BEFORE this process imports torch (the parent never touches the
GPU), env:// rendezvous on 127.0.0.1 and a free port, rank 0's JSON line relayed once, any
failing rank ends the whole launch non-zero.

Weak scaling: the per-GPU batch is fixed, ``value`` is the WHOLE-JOB throughput (all ranks);
the timed region is bracketed by a barrier + device synchronize on both sides and the
maximum elapsed time over ranks is used.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _maybe_self_launch() -> None:
    """``--gpus N > 1`` outside torchrun: run N ranks of this script and exit with their verdict.
    Runs before ``import torch``; the launcher module is loaded by path so that the grace_amd
    package (which imports torch) is not imported in the parent either."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    pre.add_argument("--launch-timeout", type=float, default=3000.0)
    a, _ = pre.parse_known_args()
    if a.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    import importlib.util

    spec = importlib.util.spec_from_file_location("_grace_launcher", os.path.join(ROOT, "grace_amd", "launcher.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    cmd = [sys.executable, "-u", os.path.abspath(__file__), *sys.argv[1:]]
    sys.exit(mod.launch(cmd, a.gpus, timeout_s=a.launch_timeout))


if __name__ == "__main__":
    _maybe_self_launch()

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HEADLINE_METRIC = "images/sec (whole node) ResNet-50 Top-K 1% @ 1/2/4/8 MI355X; comm wall-time"

# Published reference numbers in the metric's unit.  The reference publishes none for its GRACE
# harness; its only number is cifar10-fast ResNet-9: 24 epochs x 50 000 images in
# 74 s of DAWNBench train time on one V100 (examples/dist/CIFAR10-dawndist/README.md:17, 24-26).
REFERENCE_VALUE = {"resnet9_dawn": 24 * 50000 / 74.0}


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); N > 1 without torchrun's WORLD_SIZE self-launches N ranks")
    ap.add_argument("--launch-timeout", type=float, default=3000.0,
                    help="self-launch only: kill every rank after this many seconds (exit 124)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="resnet50_topk")
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (0 = workload default)")
    ap.add_argument("--bucket-mb", type=float, default=128.0,
                    help="GRACE bucket cap; 128 MB = one bucket for ResNet-50 (measured fp32 Top-K: 13.23 ms/step "
                         "vs 13.33 with 64 MB / 13.83 with 25 MB + overlap; profiles/r2_overlap_buckets.txt)")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32",
                    help="compute dtype; fp32 (default) = the reference harness's precision "
                         "(pytorch_synthetic_benchmark.py:86,151-160: plain model(data), no autocast, "
                         "TF32/xf32 disabled); bf16 = autocast, an explicitly labelled secondary run")
    ap.add_argument("--overlap", choices=["auto", "on", "off"], default="auto",
                    help="compress+communicate on a side stream during backward; auto = under a "
                         "whole-step HIP graph on only when the estimated dense exchange exceeds the ~0.9 ms "
                         "forked-capture cost (never for the compressed pipelines), on otherwise")
    ap.add_argument("--no-overlap", action="store_true", help="same as --overlap off")
    ap.add_argument("--bf16-weights", choices=["on", "off"], default="on",
                    help="fp32 master weights + bf16 working copies of conv/linear weights (autocast "
                         "numerics without the per-layer cast kernels; parallel/precision.py)")
    ap.add_argument("--optimizer", choices=["fused", "torch"], default="fused",
                    help="fused: grace_amd FusedSGD (one native multi-tensor kernel that also writes the bf16 "
                         "working copies); torch: torch.optim.SGD (foreach)")
    ap.add_argument("--grad-mode", choices=["gather", "accumulate"], default="gather",
                    help="gather: zero_grad(set_to_none) + one native gather launch per bucket; "
                         "accumulate: bucket memset + AccumulateGrad adds into bucket views")
    ap.add_argument("--no-benchmark-mode", action="store_true", help="disable MIOpen find (cudnn.benchmark)")
    ap.add_argument("--exposed-steps", type=int, default=3,
                    help="untimed eager steps after the timed region: GraceProfiler split of the exchange "
                         "(compress / comm / decompress ms, bytes on the wire) and the exposed exchange time")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise the RCCL process group even for one GPU (exercises the collective path)")
    ap.add_argument("--graph", choices=["auto", "full", "compute", "off"], default="auto",
                    help="HIP graphs: full = whole step (fwd+bwd+GRACE+RCCL+optimizer) captured; compute = "
                         "forward+backward graphed, GRACE + optimizer eager; auto = full for graph-safe "
                         "GRACE pipelines (any world size), eager otherwise")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process group: nccl = RCCL over xGMI (one GPU per rank); gloo = host transport, lets "
                         "several ranks share one GPU (multi-rank rehearsal on a 1-GPU box; --comm torch, no "
                         "whole-step graph: gloo collectives are not capturable)")
    ap.add_argument("--grace-split", choices=["on", "off"], default="on",
                    help="after the timed region, replay the measured whole-step graph interleaved with the same "
                         "step whose GRACE exchange is a no-op (None compressor, local comm: a copy) and report "
                         "the mean paired difference +- 95 %% CI as grace_ms_per_step (compress + collective + "
                         "decode as the measured step pays it)")
    ap.add_argument("--surface", choices=["engine", "ddp"], default="engine",
                    help="engine: grace_amd DistributedOptimizer (bucketed GRACE engine, the default); ddp: "
                         "torch DistributedDataParallel + grace_comm_hook (the DDP comm-hook surface; DDP owns "
                         "bucketing and backward overlap; eager unless --graph full)")
    ap.add_argument("--comm", choices=["auto", "torch", "native", "native-inline", "xgmi"], default="auto",
                    help="collective runtime: torch = ProcessGroupNCCL (RCCL, its own stream: an event "
                         "fork/join per collective); native = grace_amd RCCL runtime on its comm stream; "
                         "native-inline = grace_amd RCCL runtime on the CURRENT stream; auto = native-inline "
                         "under a whole-step graph without overlap (measured 0.44 ms/step less than torch "
                         "for ResNet-50 Top-K), torch otherwise; xgmi = native-inline plus the one-shot "
                         "peer-memory all-gather for payloads <= 8 MB (parallel/xgmi.py, self-checked at start)")
    ap.add_argument("--rccl-ctas", default="auto",
                    help="workgroup (channel) budget of the native RCCL communicator, ncclConfig_t minCTAs/maxCTAs: "
                         "auto = at W > 1 for a dense all-reduce pipeline (None / FP16 + Allreduce) probe "
                         "RcclComm.CTA_CANDIDATES on the real bucket size and keep the fastest (MAX over ranks); "
                         "off = RCCL's default; 'MIN/MAX' = fixed")
    ap.add_argument("--graph-split", choices=["auto", "on", "off"], default="auto",
                    help="whole-step graph as two LINEAR graphs (critical stream / weight-gradient side stream, "
                         "flag-word sync between them) plus the post-join graph, instead of one forked graph "
                         "(parallel/graph.py GraphedStep split): ~0.3 ms of host issue per step instead of ~9; "
                         "auto = on (engine without overlap, DDP with the deferred hook)")
    ap.add_argument("--tail-bucket", choices=["on", "off"], default="off",
                    help="engine: the first layer's weight (its gradient is the last one backward produces) in a "
                         "bucket of its own, exchanged last -- under split graphs the other buckets' exchange "
                         "overlaps that weight gradient on the side stream (measured neutral: the Top-K "
                         "histogram and the stem's weight-gradient GEMM contend, profiles/r6_graph_split.txt)")
    ap.add_argument("--ddp-defer", choices=["auto", "on", "off"], default="auto",
                    help="--surface ddp: the GRACE comm hook hands DDP its bucket back and runs the exchange "
                         "after backward (GraceHookState(defer=True)): DDP-managed weight gradients may then run "
                         "on the side stream and the step may be a split graph; auto = on under a whole-step graph")
    ap.add_argument("--deterministic", action="store_true",
                    help="bitwise-reproducible BN backward (fixed-order fp64 tree instead of atomic fp32 "
                         "totals; GRACE_BN_DETERMINISTIC=1)")
    ap.add_argument("--xgmi-capacity-mb", type=float, default=8.0,
                    help="per-rank payload capacity of the xGMI one-shot comm (two slots of this size are exported "
                         "per rank); collectives above it go to RCCL / the inner comm")
    return ap.parse_args()


def _grace_split(args, run, opt, base_opt, named, weights, w, model, data, amp, set_to_none, world, dev):
    """GRACE's cost inside the measured whole-step graph, MEASURED by interleaving: the same step
    is captured a second time with the GRACE exchange replaced by a no-op (None compressor + a
    local comm = one copy per bucket), and the two graphs are replayed ALTERNATELY, each replay
    bracketed by device events on the stream.  Every pair (measured_i, no-op_i) runs under the
    same clocks / thermals, so the paired difference d_i = measured_i - no-op_i is the exchange's
    cost (compress + collective + decode as the graphed step pays it) without the box-drift noise
    of two separately timed runs.  Returns (mean d, 95 % CI half-width,
    mean no-op ms, pairs); MAX over ranks for W > 1."""
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer
    from grace_amd.parallel.comm import LocalComm
    from grace_amd.parallel.graph import GraphedStep

    opt.engine.remove()  # the measured engine's hooks must not fire in the no-op graph
    noop = DistributedOptimizer(base_opt, grace_from_params({"compressor": "none", "communicator": "allreduce"},
                                                            comm=LocalComm()),
                                named_parameters=named, bucket_cap_mb=args.bucket_mb, overlap=False,
                                weights=weights, tail_bucket=args.tail_bucket == "on")

    def noop_step():
        noop.zero_grad(set_to_none=set_to_none)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp, cache_enabled=False):
            l3 = w.loss(model, data)
        l3.backward()
        noop.step()
        return l3

    run2 = GraphedStep(noop_step, warmup=3, split=getattr(run, "split", False))
    for _ in range(3):
        run(), run2()
    torch.cuda.synchronize()
    pairs = max(10, 2 * args.steps)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * pairs + 1)]
    ev[0].record()
    for i in range(pairs):
        run()
        ev[2 * i + 1].record()
        run2()
        ev[2 * i + 2].record()
    torch.cuda.synchronize()
    a = [ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(pairs)]
    b = [ev[2 * i + 1].elapsed_time(ev[2 * i + 2]) for i in range(pairs)]
    d = [x - y for x, y in zip(a, b)]
    mean = sum(d) / pairs
    sd = (sum((v - mean) ** 2 for v in d) / max(1, pairs - 1)) ** 0.5
    ci = 1.96 * sd / pairs ** 0.5
    t = torch.tensor([mean, ci, sum(b) / pairs], dtype=torch.float64, device=dev)
    if world > 1:
        if args.backend == "gloo":
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    mean, ci, noop_ms = (float(v) for v in t.tolist())
    return mean, ci, noop_ms, pairs


def _dense_bucket_payload(w, model, bucket_mb: float) -> int:
    """Bytes one dense bucket puts on the wire: the engine fills fp32 buckets of ``bucket_mb``
    (the last one partial), the FP16 compressor then halves each bucket's payload (ADVICE r5:
    probe and bucket count in the same units)."""
    esz = 2 if w.grace.get("compressor") == "fp16" else 4
    fp32_bucket = min(sum(p.numel() for p in model.parameters()) * 4, int(bucket_mb * 2 ** 20))
    return fp32_bucket * esz // 4


def _rccl_nranks(rccl_obj, world_seen: int, gloo: bool):
    """What the communicators report: the native RCCL runtime's own ncclCommCount (and the device
    RCCL bound) when GRACE traffic runs on it, the torch process group's size otherwise."""
    out = {"process_group": world_seen if not gloo else None}
    if rccl_obj is not None:
        try:
            out["native_rccl"] = rccl_obj.nranks
            out["native_rccl_device"] = rccl_obj.comm_device
        except Exception as e:  # noqa: BLE001 -- reporting only
            out["native_rccl"] = f"unavailable: {type(e).__name__}"
    return out


def main() -> int:
    args = parse()
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer, broadcast_parameters
    from grace_amd.utils.workloads import WORKLOADS, build_model

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: a torchrun launch must pass --gpus WORLD_SIZE")
    if args.deterministic:
        os.environ["GRACE_BN_DETERMINISTIC"] = "1"  # read when the BN ops are first used
    ndev = torch.cuda.device_count()  # counting devices does not initialise the GPU
    gloo = args.backend == "gloo"
    if not gloo and local >= ndev:
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {ndev} visible GPU(s); RCCL needs one GPU per "
                         f"rank (--backend gloo lets ranks share a GPU for a rehearsal)")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    if gloo:  # ranks may share GPUs
        local = local % ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if args.surface == "ddp":
        args.force_dist = True  # DDP needs a process group even for one rank
    if world > 1 or args.force_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        if gloo:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)  # RCCL over xGMI
    torch.backends.cudnn.benchmark = not args.no_benchmark_mode
    # strict fp32: no reduced-precision (xf32) conv/GEMM paths
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False

    w = WORKLOADS[args.workload]
    batch = args.batch or w.batch
    torch.manual_seed(0)
    model = build_model(w, dev)
    broadcast_parameters(model.state_dict(), root_rank=0)
    weights = None
    named = list(model.named_parameters())
    if args.bf16_weights == "on" and args.dtype == "bf16":
        from grace_amd.parallel.precision import BF16Weights

        weights = BF16Weights(model)
        named = list(weights.named_master_parameters(model))
    if args.optimizer == "fused":
        from grace_amd.parallel import FusedSGD

        base_opt = FusedSGD([p for _, p in named], lr=0.01 * world, momentum=0.5)
    else:
        base_opt = torch.optim.SGD([p for _, p in named], lr=0.01 * world, momentum=0.5)
    from grace_amd.parallel.graph import GraphedStep, graph_compute, graph_safe

    mode = args.graph
    # a gloo group cannot capture its collectives, but an ALL-GATHER-only pipeline's exchange can
    # run on the xGMI one-shot comm (peer memory, gloo only bootstraps it): that is the W > 1
    # whole-step-graph rehearsal on a 1-GPU box (ranks share the card)
    # (every Allgather / Allreduce pipeline: XgmiComm gathers one-shot, all-reduces by a one-shot
    # gather + rank-ordered local reduction -- PowerSGD's P / Q, DGC's clipping norm, the dense
    # buckets -- and runs QSGD's compressed-domain all-to-all one-shot, all while the payload fits
    # --xgmi-capacity-mb; tests/test_gpu_xgmi.py checks each against an eager W = 2 run)
    gloo_graph = (gloo and world > 1 and args.comm in ("xgmi", "auto") and args.surface == "engine"
                  and w.grace.get("communicator") in ("allgather", "allreduce"))
    if args.surface == "ddp" and mode == "auto":
        # the whole DDP step (reducer + comm hook) captures: 2341 vs 2309 img/s eager
        # (profiles/r3_ddp_surface.txt); a failed capture falls back to eager below
        mode = "off" if (gloo and world > 1) else "full"
    if mode == "auto":
        # measured on MI355X (ResNet-50 Top-K 1%): full 3205 img/s, compute 2640, eager 2520-3240
        # (eager is host-launch bound: ~1100 kernels per step); full without overlap 3525
        probe = grace_from_params(dict(w.grace, world_size=world))
        mode = "full" if graph_safe(probe) is None else "off"
        del probe
        if gloo and world > 1 and not (gloo_graph and mode == "full"):
            mode = "compute"  # gloo collectives cannot be captured
    if gloo and world > 1 and mode == "full" and not gloo_graph:
        raise SystemExit("--graph full with gloo needs an all-gather-only pipeline and --comm xgmi/auto "
                         "(the exchange on the xGMI one-shot comm); else use --backend nccl")
    if args.no_overlap:
        args.overlap = "off"
    # --overlap auto under the whole-step graph: on only when the exchange could hide more than a
    # forked capture costs.  Fork cost: ~0.9 ms/step for ResNet-50 (profiles/r2_overlap_buckets.txt).
    # Exchange time: MEASURED for the dense pipelines -- the RCCL channel-budget probe
    # (RcclComm.tuned, run here ahead of the decision) all-reduces the real bucket on the real links
    # and its best time (MAX over ranks) is the exchange the fork could hide; every compressed
    # pipeline's exchange is a few-MB gather: off.  (The W = 2 rehearsal with two ranks SHARING one
    # GPU, profiles/r4_overlap_w2_rehearsal.txt, measures the shared card, not links.)
    dense_ar = w.grace.get("communicator") == "allreduce" and w.grace.get("compressor") in ("none", "fp16")
    rccl_pre = None
    overlap_note = None
    if (world > 1 and not gloo and dense_ar and args.rccl_ctas == "auto" and args.surface == "engine"
            and mode == "full" and args.comm in ("auto", "native", "native-inline", "xgmi")):
        from grace_amd.parallel.native_comm import RcclComm

        nbytes = _dense_bucket_payload(w, model, args.bucket_mb)
        try:
            rccl_pre = RcclComm.tuned(nbytes)  # collective: every rank builds / probes the candidates
        except Exception as e:  # noqa: BLE001 -- e.g. no ncclConfig support: keep the default comm
            print(f"[rank {rank}] RCCL CTA probe failed ({type(e).__name__}: {str(e)[:120]}); default channels",
                  file=sys.stderr, flush=True)
            rccl_pre = None
        ok_t = torch.tensor([0 if rccl_pre is None else 1], device=dev)
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)  # every rank keeps the probe, or none does
        if ok_t.item() == 0:
            rccl_pre = None
    if args.overlap == "auto" and mode == "full" and world > 1:
        est_ms = 0.0
        if rccl_pre is not None:
            n_buckets = max(1, -(-sum(p.numel() for p in model.parameters()) * 4 // int(args.bucket_mb * 2 ** 20)))
            est_ms = min(rccl_pre.choice["us"].values()) * n_buckets / 1e3
            overlap_note = f"measured dense all-reduce {est_ms:.3f} ms/step vs ~0.9 ms forked-capture cost"
        args.overlap = "on" if est_ms > 0.9 else "off"
    overlap = args.overlap == "on" or (args.overlap == "auto" and mode != "full")
    comm_kind = "local"
    comm_obj = None
    rccl_obj = None
    xgmi_note = None
    if dist.is_initialized():
        comm_kind = args.comm
        if comm_kind == "auto":
            # whole-step graph without overlap: the in-line native RCCL runtime, wrapped by the
            # xGMI one-shot comm whose all-gathers pick their path per payload size by a start-up
            # MEASUREMENT against RCCL's (MAX over ranks; XgmiComm select="probe"); a box where
            # the peer mapping fails keeps plain RCCL
            comm_kind = "auto-probe" if (mode == "full" and not overlap) else "torch"
        if gloo:
            comm_kind = ("xgmi" if args.comm == "xgmi" else "auto-probe") if (gloo_graph and mode == "full") \
                else "torch"
        if comm_kind != "torch":
            from grace_amd.parallel import set_default_comm
            from grace_amd.parallel.native_comm import RcclComm

            try:
                if gloo:
                    from grace_amd.parallel.comm import TorchComm

                    native = TorchComm()
                else:
                    inl = comm_kind in ("native-inline", "xgmi", "auto-probe")
                    if rccl_pre is not None:  # probed above (the overlap decision used its time)
                        rccl_pre.set_inline(inl)
                        native = rccl_pre
                    elif args.rccl_ctas == "auto" and world > 1 and dense_ar:
                        # the dense all-reduce's channel budget for the 7-link mesh, measured on the
                        # real bucket: one ring drives one outbound link per GPU
                        native = RcclComm.tuned(_dense_bucket_payload(w, model, args.bucket_mb), inline=inl)
                    else:
                        ctas = (0, 0) if args.rccl_ctas in ("auto", "off") else \
                            tuple(int(v) for v in args.rccl_ctas.split("/"))
                        native = RcclComm.from_process_group(inline=inl, ctas=ctas)
                    rccl_obj = native
                if comm_kind in ("xgmi", "auto-probe"):
                    from grace_amd.parallel.xgmi import XgmiComm

                    try:
                        # construction verifies the one-shot gather (staged and from the exported
                        # slot) and all-to-all bit-exactly against the inner comm on every rank
                        native = XgmiComm(native, capacity_mb=args.xgmi_capacity_mb,
                                          select="probe" if comm_kind == "auto-probe" else "size")
                        xgmi_note = {"verified_vs_inner": True, "inner": type(native.inner).__name__,
                                     "direct_slot": bool(native._direct_ok)}
                    except Exception as e:  # every rank raised together (XgmiComm agrees)
                        if comm_kind == "xgmi" or gloo:
                            raise
                        print(f"[rank {rank}] xGMI one-shot comm unavailable ({str(e)[:120]}); RCCL only",
                              file=sys.stderr, flush=True)
                        comm_kind = "native-inline (xgmi setup failed)"
                        xgmi_note = {"verified_vs_inner": False, "fallback": "RCCL on every rank",
                                     "error": str(e)[:200]}
                comm_obj = native
                ok = 1
            except Exception as e:  # every rank must agree before the first GRACE collective
                print(f"[rank {rank}] native RCCL comm unavailable ({type(e).__name__}: {str(e)[:120]}); "
                      f"using torch.distributed", file=sys.stderr, flush=True)
                native, ok = None, 0
            flag = torch.tensor([ok], device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if flag.item() == 1:
                set_default_comm(native)
            else:
                comm_kind = "torch (native comm failed)"
    grc = grace_from_params(dict(w.grace, world_size=world))
    # split graphs (critical stream A / side stream B / A2; see the capture below) unless the step
    # overlaps its exchange with backward or DDP's hook runs immediately
    ddp_defer = args.ddp_defer == "on" or (args.ddp_defer == "auto" and mode == "full")
    # (never with overlap or an immediate DDP hook, --graph-split on included: the side stream must
    # then be joined on the capture stream after backward)
    split_planned = (mode == "full" and args.graph_split != "off" and not overlap
                     and not (args.surface == "ddp" and not ddp_defer))
    main_stream = None
    if split_planned:
        # A and B must sit on DIFFERENT hardware queues: HIP deals streams of one priority to a few
        # HW queues (GPU_MAX_HW_QUEUES, 4), and once the native RCCL runtime had created its
        # streams the side stream shared the replay stream's queue -- the two graphs serialised
        # (2494-2515 img/s at W = 1 vs 2746-2752 with the step on a high-priority stream, whose
        # queue pool holds nothing else; profiles/r6_graph_split.txt)
        from grace_amd.ops.wgrad import dedicated_stream

        main_stream = dedicated_stream(local, -1, "bench-main")
        main_stream.wait_stream(torch.cuda.current_stream(dev))
        torch.cuda.set_stream(main_stream)
    ddp_state = ddp_stream = None
    if args.surface == "ddp":
        from grace_amd.parallel import GraceHookState, grace_comm_hook

        if weights is not None:
            raise SystemExit("--surface ddp trains fp32 masters directly (use --bf16-weights off)")
        # buffers (BN running statistics) are broadcast once at start like the engine path and the
        # reference's Horovod harness, not before every forward
        # a captured DDP step: the reducer's AccumulateGrad nodes take the stream current at
        # construction, so build DDP under the stream the step is captured and replayed on
        ddp_stream = (main_stream if main_stream is not None else torch.cuda.Stream(dev)) if mode == "full" else None
        with torch.cuda.stream(ddp_stream) if ddp_stream is not None else contextlib.nullcontext():
            model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local], bucket_cap_mb=args.bucket_mb,
                                                              gradient_as_bucket_view=True, broadcast_buffers=False)
        # deferred hook where the step becomes split graphs (a forked DDP graph is host-bound:
        # 2352 vs 2468 img/s immediate)
        ddp_state = GraceHookState(grc, model=model, defer=ddp_defer)
        model.register_comm_hook(ddp_state, grace_comm_hook)
        if ddp_stream is not None and hasattr(torch.autograd.graph, "set_warn_on_accumulate_grad_stream_mismatch"):
            # intentional: DDP's reducer keeps AccumulateGrad nodes created on the capture stream (see
            # above), so the eager warm-up steps before the capture run them across streams
            torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)

        class _DdpOpt:  # the bench loop's optimizer interface over DDP + a plain optimizer
            engine = type("E", (), {"grc": grc})()

            def zero_grad(self, set_to_none=True):
                base_opt.zero_grad(set_to_none=set_to_none)

            def step(self):
                ddp_state.flush()  # the deferred GRACE exchange (no-op for the immediate hook)
                base_opt.step()

            def abort_step(self):
                pass

        opt = _DdpOpt()
    else:
        opt = DistributedOptimizer(base_opt, grc, named_parameters=named,
                                   bucket_cap_mb=args.bucket_mb, overlap=overlap, weights=weights,
                                   tail_bucket=args.tail_bucket == "on")
    data = w.make_batch(batch, dev)
    if w.channels_last and isinstance(data, tuple) and data[0].dim() == 4:
        data = (data[0].contiguous(memory_format=torch.channels_last),) + tuple(data[1:])
    amp = args.dtype == "bf16"

    fwd_model = model

    set_to_none = args.grad_mode == "gather"

    def step():
        opt.zero_grad(set_to_none=set_to_none)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp, cache_enabled=False):
            loss = w.loss(fwd_model, data)
        loss.backward()
        opt.step()
        return loss

    if mode == "compute" and not (isinstance(data, tuple) and data[0].is_floating_point()):
        mode = "off"  # token-input models: graph only with the full-step capture
    graph_note = "off"
    run = step
    try:
        if mode == "full":
            # DDP records runtime-logging events (and reads them back with a host sync) in its
            # first 10 iterations: capture only after those
            cap_warm = max(3, args.warmup // 2) if args.surface == "engine" else max(11, args.warmup)
            # split graphs (critical / side stream, flag sync every 2 fork points): 2730-2750 img/s
            # at 0.2 ms of host issue vs the forked graph's 2700-2720 at 9.2 ms, also with the native
            # RCCL runtime in the step (--force-dist); DDP (deferred hook) 0.99 of the engine; W = 2
            # sharing one GPU 3104 vs 2463 (profiles/r6_graph_split.txt).  Forked: overlap, or an
            # immediate DDP hook (the side stream must be joined on the capture stream after backward)
            split = split_planned
            run = GraphedStep(step, warmup=cap_warm, stream=ddp_stream,
                              capture_error_mode="thread_local" if world > 1 else None, split=split)
            graph_note = "full (split: A / side B / A2)" if run.split else "full"
        elif mode == "compute":
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp, cache_enabled=False):
                fwd_model = graph_compute(model, data[0], engine=opt.engine)
            graph_note = "compute"
    except Exception as e:  # capture unsupported -> stay eager
        import traceback

        traceback.print_exc(file=sys.stderr)
        graph_note = f"failed: {type(e).__name__}: {str(e)[:120]}"
        torch.cuda.synchronize()
        opt.abort_step()  # a capture that raised mid-backward leaves buckets half launched
        fwd_model, run = model, step
    if dist.is_initialized():  # every rank must run the same mode (collective sequences must match)
        ok = torch.tensor([0 if graph_note.startswith("failed") else 1], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if ok.item() == 0 and not graph_note.startswith("failed"):
            graph_note, fwd_model, run = "off (a peer failed to capture)", model, step

    def barrier():
        if world > 1:
            if gloo:
                dist.barrier()
            else:
                dist.barrier(device_ids=[local])

    trace_loss = os.environ.get("GRACE_BENCH_LOSS_TRACE", "0") == "1"  # debug: per-step loss to stderr
    # debug: every step's loss copied on the device (no host sync between steps), printed at the end
    rec = torch.empty(args.warmup + args.steps, device=dev) \
        if os.environ.get("GRACE_BENCH_LOSS_RECORD", "0") == "1" else None
    for i in range(args.warmup):
        lw = run()
        if rec is not None:
            rec[i].copy_(lw.float().reshape(()))
        if trace_loss:
            print(f"[bench] warmup step {i} loss {float(lw.float().item()):.5f}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    # per-step device events (recorded on the stream, no host sync inside the timed region) give
    # the reference harness's statistic: mean +- 1.96 std of img/s (pytorch_synthetic_benchmark.py:182-198)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(args.steps):
        loss = run()
        evs[i + 1].record()
        if rec is not None:
            rec[args.warmup + i].copy_(loss.float().reshape(()))
        if trace_loss:
            print(f"[bench] timed step {i} loss {float(loss.float().item()):.5f}", file=sys.stderr, flush=True)
    issue_s = time.perf_counter() - t0  # host time to issue the steps (graph replays) before the wait
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # a device-side communication fault inside the timed replays (an xGMI peer wait that timed
    # out: FusedSGD skipped those updates) or an RCCL async error must fail the run loudly
    from grace_amd.parallel import health as _health

    _health.check()
    _chk = getattr(opt.engine.grc.comm, "check", None)
    if callable(_chk):
        _chk()
    step_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
    if os.environ.get("GRACE_GRAPH_CENSUS", "0") == "1" and hasattr(run, "graphs"):
        from grace_amd.ops import _native as _nat

        names = ("kernel", "memcpy", "memset", "host", "graph", "empty", "wait_event", "event_record",
                 "sem_signal", "sem_wait", "mem_alloc", "mem_free", "t12", "t13", "t14")
        for tag, g in (("A", run.graphs[0]), ("B", getattr(run, "g_side", None)), ("A2", getattr(run, "g_a2", None))):
            if g is not None:
                c = _nat.lib().graph_node_types(g.raw_cuda_graph())
                print(f"[graph-census] {tag}: " + " ".join(f"{n}={c[i]}" for i, n in enumerate(names) if c[i])
                      + f" multi_dep={c[15]}", file=sys.stderr)
    if os.environ.get("GRACE_SPLIT_TRACE", "0") == "1" and getattr(run, "split", False):
        for row in run._sc.timeline():  # (fork, A signalled us, B's wait returned us, lag us)
            print("[split-trace] fork %3s  A %9.1f  B %9.1f  lag %8.1f" % row, file=sys.stderr)
    if rec is not None:
        print("[bench] losses " + " ".join(f"{v:.4f}" for v in rec.tolist()), file=sys.stderr, flush=True)
    final_loss = float(loss.float().item())
    loss_finite = final_loss == final_loss and abs(final_loss) != float("inf")
    if not loss_finite:  # a diverged run's throughput is not a measurement of training
        print(f"[rank {rank}] ERROR: final loss is {final_loss}: the timed steps trained a diverged model; "
              f"the throughput below is NOT a valid {w.name} number", file=sys.stderr, flush=True)
    # every rank's own timed-region wall time (the spread shows a straggler); the MAX is the job's
    per_rank_s = [elapsed]
    if world > 1:
        el_dev = torch.device("cpu") if gloo else dev
        mine = torch.tensor([elapsed], dtype=torch.float64, device=el_dev)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank_s = [float(t.item()) for t in allr]
    elapsed = max(per_rank_s)
    world_seen = dist.get_world_size() if dist.is_initialized() else 1

    # untimed: the reference harness's "comm wall-time" split (pytorch_synthetic_benchmark.py:
    # 166-167) -- eager steps with the GraceProfiler attached: compress (compensate + compress +
    # residual update), comm (collective issue -> completion as seen by the consuming stream),
    # decompress (decode + aggregate into the bucket), bytes on the wire per rank; plus the
    # EXPOSED exchange time: opt.step() (exchange + optimizer) after a fully synchronised backward
    from grace_amd.utils.profiler import GraceProfiler

    prof = GraceProfiler(roctx=False)
    opt.engine.grc.profiler = prof
    exposed = []
    for i in range(args.exposed_steps):
        opt.zero_grad(set_to_none=set_to_none)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp, cache_enabled=False):
            l2 = w.loss(fwd_model, data)
        if i == 0:
            prof.reset()
        l2.backward()
        torch.cuda.synchronize()
        barrier()
        t = time.perf_counter()
        opt.step()
        torch.cuda.synchronize()
        exposed.append(time.perf_counter() - t)
        prof.step()
    opt.engine.grc.profiler = None
    # drop the eager steps' autograd graph: it keeps the parameters' AccumulateGrad nodes alive,
    # bound to THIS stream, and a later capture (the no-op graph below) on another stream would
    # run them outside the capture ("capturing stream has unjoined work")
    l2 = None  # noqa: F841
    split = prof.report() if args.exposed_steps else {}
    ex = torch.tensor([sum(exposed) / max(1, len(exposed))], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ex, op=dist.ReduceOp.MAX)

    # GRACE's cost inside the measured path: paired, interleaved replays of the measured graph and
    # the same step with a no-op exchange (_grace_split); diagnostics only, after the timed region
    grace_ms = grace_ci = grace_raw = noop_ms = grace_pairs = None
    grace_split_note = None
    if args.grace_split == "on" and graph_note.startswith("full") and args.surface == "engine":
        try:  # a failure here must not cost the measured line
            grace_raw, grace_ci, noop_ms, grace_pairs = _grace_split(
                args, run, opt, base_opt, named, weights, w, model, data, amp, set_to_none, world, dev)
            # a cost is not negative: a pipeline whose exchange IS the no-op (None at W = 1) reads
            # 0 within its CI; grace_ms_raw keeps the signed mean
            grace_ms = max(0.0, grace_raw)
        except Exception as e:  # noqa: BLE001
            grace_split_note = f"no-op graph failed: {type(e).__name__}: {str(e)[:100]}"
            print(f"[rank {rank}] grace split skipped ({grace_split_note})", file=sys.stderr, flush=True)
            try:
                torch.cuda.synchronize()
            except Exception:  # noqa: BLE001
                pass

    samples = w.samples_per_batch(batch) * world * args.steps
    value = samples / elapsed if loss_finite else None  # a diverged run reports no throughput
    per_gpu = [w.samples_per_batch(batch) / (ms * 1e-3) for ms in step_ms if ms > 0]
    mean_pg = sum(per_gpu) / max(1, len(per_gpu))
    std_pg = (sum((v - mean_pg) ** 2 for v in per_gpu) / max(1, len(per_gpu))) ** 0.5
    if rank == 0:
        metric = HEADLINE_METRIC if w.name == "resnet50_topk" else f"{w.unit}/sec (whole node) {w.name}"
        out = {
            "metric": metric,
            "value": None if value is None else round(value, 2),
            "unit": f"{w.unit}/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / REFERENCE_VALUE[w.name], 3)
            if (w.name in REFERENCE_VALUE and value is not None) else None,
            "dtype": args.dtype,
            "data": "synthetic (random-init weights)",
            "config": {
                "model": w.model,
                "global_batch": batch * world,
                "per_gpu_batch": batch,
                "seq_len": w.seq_len,
                "parallelism": f"dp{world}",
                "backend": ("gloo (ranks share GPUs: rehearsal, not a scaling number)" if gloo else "nccl (RCCL)")
                if dist.is_initialized() else "none (W=1, no process group: local comm)",
                "grace": w.grace,
                "bucket_mb": args.bucket_mb,
                "buckets": len(opt.engine.buckets) if hasattr(opt.engine, "buckets") else None,
                "overlap": overlap,
                **({"overlap_rule": overlap_note} if overlap_note else {}),
                "hip_graph": graph_note,
                "comm": comm_kind,
                "grad_mode": args.grad_mode,
                "surface": args.surface + (f" ({len(ddp_state.layouts)} DDP buckets, "
                                           f"{'deferred' if ddp_state.defer else 'immediate'} hook)" if ddp_state else ""),
                "bf16_weights": weights is not None,
                "optimizer": f"{'FusedSGD' if args.optimizer == 'fused' else 'torch.optim.SGD'}(lr={0.01 * world:g}, momentum=0.5)",
            },
            "per_gpu": {"mean": round(mean_pg, 2), "ci95": round(1.96 * std_pg, 2),
                        "note": f"{w.unit}/sec per GPU on rank 0, mean +- 1.96 std over {len(per_gpu)} steps"},
            "exchange_ms": dict({k.replace("_ms_per_step", ""): round(v, 4) for k, v in split.items()
                                 if k.endswith("_ms_per_step")},
                                **({} if dist.is_initialized() else
                                   {"note": "W=1 without a process group: 'comm' is a local device copy, "
                                            "not a collective"})),
            "comm_choice": (list(getattr(comm_obj, "choices", {}).values()) or None) if comm_obj is not None else None,
            "world_seen": world_seen,
            "rccl_nranks": _rccl_nranks(rccl_obj, world_seen, gloo),
            "per_rank_ms_per_step": {"min": round(min(per_rank_s) / args.steps * 1e3, 3),
                                     "max": round(max(per_rank_s) / args.steps * 1e3, 3),
                                     "ranks": len(per_rank_s)},
            "xgmi": xgmi_note,
            "rccl_ctas": (getattr(rccl_obj, "choice", None) or {"ctas": list(getattr(rccl_obj, "ctas", (0, 0)))})
            if rccl_obj is not None else None,
            "bn_backward": ("fixed-order fp64 tree (deterministic)" if os.environ.get("GRACE_BN_DETERMINISTIC") == "1"
                            else "atomic fp32 totals (run-to-run order noise ~1e-7 rel.; GRACE_BN_DETERMINISTIC=1 "
                                 "for bitwise reproducibility)"),
            "bytes_on_wire_per_rank": int(split.get("bytes_per_step", 0)),
            "grace_ms_per_step": None if grace_ms is None else round(grace_ms, 3),
            "grace_ms_ci95": None if grace_ci is None else round(grace_ci, 3),
            "grace_ms_raw": None if grace_raw is None else round(grace_raw, 4),
            "grace_split": None if grace_pairs is None else
            f"mean of {grace_pairs} paired differences (measured graph replay - no-op-exchange graph replay, "
            f"interleaved, device events), +- 95 % CI; MAX over ranks",
            **({"grace_split_note": grace_split_note} if grace_split_note else {}),
            "noop_exchange_ms_per_step": None if noop_ms is None else round(noop_ms, 3),
            "exposed_exchange_ms_eager": round(float(ex.item()) * 1e3, 3),
            "host_issue_ms_per_step": round(issue_s / args.steps * 1e3, 3),
            "final_loss": round(final_loss, 4) if loss_finite else str(final_loss),
            "loss_finite": loss_finite,
        }
        print(json.dumps(out), flush=True)
        if os.environ.get("GRACE_AUTOTUNE_REPORT", "0") == "1":  # the per-layer backend choices, to stderr
            from grace_amd.ops import conv as _cv

            for row in _cv.autotune_table():
                print("conv1x1", row[:5], {k: round(v, 4) for k, v in row[5].items()}, file=sys.stderr)
            for row in _cv.conv3x3_autotune_table():
                print("conv", row[:9], {k: round(v, 4) for k, v in row[9].items()}, file=sys.stderr)
            for row in _cv.bn_autotune_table():  # (key..., choice, {candidate: ms})
                print("conv_bn", row[:-1], {k: round(v, 4) for k, v in row[-1].items()}, file=sys.stderr)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0 if loss_finite else 3  # a diverged run fails the launch (no throughput recorded)


if __name__ == "__main__":
    sys.exit(main())
