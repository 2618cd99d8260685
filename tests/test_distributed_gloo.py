"""Multi-process communicator semantics on CPU (gloo, W = 2 and 3).

Every rank holds rank-specific data; results are checked against the oracle of the reference
semantics computed from ALL ranks' data, and for bit-identity across ranks (the DP invariant).
"""
import os
import sys

import pytest
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(__file__))
import oracles as O  # noqa: E402
from dist_utils import run_distributed  # noqa: E402


def _data(rank, shape=(31, 17), seed=0):
    g = torch.Generator().manual_seed(1000 * seed + rank)
    return torch.randn(*shape, generator=g)


def _same_on_all_ranks(t):
    W = dist.get_world_size()
    t = t.detach().cpu().contiguous()
    out = [torch.empty_like(t) for _ in range(W)]
    dist.all_gather(out, t)
    for o in out[1:]:
        assert torch.equal(o, out[0]), "result differs across ranks"


def _replay_mean(params, xs, name, device):
    """mean over ranks r of decompress(compress_r(x_r)) with codec objects bound to rank r."""
    from grace_amd import grace_from_params
    from grace_amd.parallel.comm import LocalComm

    dec = []
    for r, x in enumerate(xs):
        c = grace_from_params(dict(params, world_size=1), comm=LocalComm()).compressor
        c.rank = r
        payload, ctx = c.compress(x.to(device).clone(), name)
        dec.append(c.decompress(payload, ctx).cpu())
    return sum(dec) / len(xs)


def _powersgd_oracle(xs, rank, name, device):
    from grace_amd.ops import powersgd as PS
    from grace_amd.ops.randomk import fnv1a64, mix_step

    n, m = xs[0].shape
    W = len(xs)
    seed = fnv1a64(name.encode())
    if device == "cpu":
        q = PS.randn_shared(m * rank, mix_step(seed, 1), "cpu").view(m, rank)
    else:  # native: device step counter 1 mixed in on the device
        q = PS.randn_shared(m * rank, seed, device, step=torch.ones(1, dtype=torch.int64, device=device)).cpu()
        q = q.view(m, rank)
    p = sum(x @ q for x in xs) / W
    p = O.gram_schmidt(p)
    q2 = sum(x.t() @ p for x in xs) / W
    return p @ q2.t()


def _body(rank, world, device="cpu"):
    """Every communicator x compressor pairing on W ranks.  device="cuda": each rank's tensors on
    cuda:0 (native HIP kernels, gloo moving the GPU payloads) -- tests/test_gpu_multirank.py."""
    from grace_amd import grace_from_params

    xs = [_data(r) for r in range(world)]
    x = xs[rank].to(device)

    def run(params, name="w"):
        p = dict(params, world_size=world)
        grc = grace_from_params(p)
        out = grc.step(x.clone(), name)
        assert out.device.type == torch.device(device).type
        _same_on_all_ranks(out)
        return out.cpu()

    # None: allreduce / allgather / broadcast all give the mean
    mean = sum(xs) / world
    for comm in ("allreduce", "allgather", "broadcast"):
        torch.testing.assert_close(run({"compressor": "none", "communicator": comm}), mean)
    # FP16
    torch.testing.assert_close(run({"compressor": "fp16", "communicator": "allreduce"}), mean, rtol=2e-3, atol=2e-3)
    # Top-K via allgather and broadcast: mean of per-rank top-k
    exp = sum(O.topk(t, 0.1) for t in xs) / world
    for comm in ("allgather", "broadcast"):
        torch.testing.assert_close(run({"compressor": "topk", "compress_ratio": 0.1, "communicator": comm}), exp)
    # Threshold (variable size) via allgather
    exp = sum(O.threshold(t, 0.8) for t in xs) / world
    torch.testing.assert_close(run({"compressor": "threshold", "threshold": 0.8, "communicator": "allgather"}), exp)
    # Random-K: identical indices on all ranks -> allreduce == allgather
    a = run({"compressor": "randomk", "compress_ratio": 0.2, "communicator": "allreduce"}, "rk")
    b = run({"compressor": "randomk", "compress_ratio": 0.2, "communicator": "allgather"}, "rk")
    torch.testing.assert_close(a, b)
    nz = a != 0
    torch.testing.assert_close(a[nz], mean[nz])
    # SignSGD majority vote (allgather and "bit-packed allreduce")
    exp = O.signsgd_vote(xs)
    torch.testing.assert_close(run({"compressor": "signsgd", "communicator": "allgather"}), exp)
    torch.testing.assert_close(run({"compressor": "signsgd", "communicator": "allreduce"}), exp)
    # EF-SignSGD: sum of mean*sign / lr
    exp = sum(O.efsign(t) for t in xs) / 0.5
    torch.testing.assert_close(run({"compressor": "efsignsgd", "lr": 0.5, "communicator": "allgather"}), exp,
                               rtol=1e-5, atol=1e-5)
    # OneBit: mean of per-rank decode
    exp = sum(O.onebit(t) for t in xs) / world
    torch.testing.assert_close(run({"compressor": "onebit", "communicator": "allgather"}), exp, rtol=1e-5, atol=1e-5)
    # QSGD shared-scale allreduce and allgather: within one quantisation step of the mean
    for comm in ("allreduce", "allgather"):
        out = run({"compressor": "qsgd", "quantum_num": 15, "communicator": comm}, "q")
        bound = max(t.norm() for t in xs) / 15
        assert (out - mean).abs().max() <= bound * (1 + 1e-4)
    # small s on the gathered path: 2-bit (s = 1) / 4-bit (s = 3) packed codes on the wire
    for s_ in (1, 3):
        out = run({"compressor": "qsgd", "quantum_num": s_, "communicator": "allgather"}, f"qp{s_}")
        assert (out - mean).abs().max() <= max(t.norm() for t in xs) / s_ * (1 + 1e-4)
    # s = 127 (BASELINE BERT config): int8 codes all-to-all + int16 level sums all-gathered
    # (compressed-domain reduce-scatter), bit-identical to the all-reduce of fp16 integer levels
    out = run({"compressor": "qsgd", "quantum_num": 127, "communicator": "allreduce"}, "q127")
    assert (out - mean).abs().max() <= max(t.norm() for t in xs) / 127 * (1 + 1e-4)
    ref = run({"compressor": "qsgd", "quantum_num": 127, "communicator": "allreduce",
               "qsgd_reduce_scatter": False}, "q127")
    assert torch.equal(out, ref)
    # TernGrad / Natural / U8bit / Sketch / INCEPTIONN / Adaq / DGC: the W-rank result equals the
    # rank-ordered average of every rank's OWN decode, replayed locally on each rank with a codec
    # object carrying that rank's id (same per-(name, rank, step) seeds as the real rank used)
    for comp in ("terngrad", "natural", "u8bit", "sketch", "inceptionn", "adaq", "dgc"):
        p = {"compressor": comp, "communicator": "allgather", "compress_ratio": 0.05}
        out = run(p, comp)
        exp = _replay_mean(p, xs, comp, device)
        torch.testing.assert_close(out, exp, rtol=1e-5, atol=1e-6)
    # PowerSGD (W-averaged P and Q, shared Q on every rank): P = mean_r(M_r Q), orthonormalised,
    # Q' = mean_r(M_r^T P); result P Q'^T (oracle with the same Q)
    out = run({"compressor": "powersgd", "compress_rank": 2, "communicator": "allreduce"}, "ps")
    exp = _powersgd_oracle(xs, 2, "ps", device)
    torch.testing.assert_close(out, exp, rtol=1e-4, atol=1e-5)
    # DGC memory with clipping (batched scalar allreduce)
    out = run({"compressor": "dgc", "memory": "dgc", "gradient_clipping": True, "communicator": "allgather",
               "compress_ratio": 0.05}, "dg")
    assert torch.isfinite(out).all()
    # Residual memory + Top-K over 3 steps keeps ranks identical
    grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.05, "memory": "residual",
                             "communicator": "allgather", "world_size": world})
    for s in range(3):
        out = grc.step(_data(rank, seed=s + 1).to(device), "w")
        _same_on_all_ranks(out)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_communicators_gloo(world):
    run_distributed(_body, world)
