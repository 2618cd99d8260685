"""Follow-up of ddp_fp64_diag.py: the first wrong gradient is the dx of layer3.0.bn2's backward
(the dual-output BN with a residual, M = 128 rows x C = 256) while the gradients handed TO that
backward are right.  This wraps the native BN forward / backward entry points, keeps copies of
every operand of that layer (forward: x, residual, save, mask, y; backward: dy, dy2, x, mask,
save, dx, dres, dweight, dbias) and checks (1) that the operands the backward reads are the ones
the forward produced and (2) the kernel's outputs against an fp64 recomputation from its inputs.
Usage: python tools/gpu/bn_bwd_capture.py --force dgrad=mfma_t2
"""
import argparse
import copy
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import ddp_fp64_diag as D  # noqa: E402
from grace_amd.ops import _native, conv  # noqa: E402

SHAPE = (8, 256, 4, 4)


VARIANT = "sync_both"


class Proxy:
    def __init__(self, real, log):
        self._real, self._log = real, log
        self.kept = []

    def __getattr__(self, k):
        return getattr(self._real, k)

    def _pin(self, t):
        """device -> pinned host copy on the current stream: no device allocation, no sync"""
        if t is None or not isinstance(t, torch.Tensor) or t.numel() == 0:
            return None
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True).as_strided(t.shape, t.stride()) \
            if t.is_contiguous() else torch.empty_like(t, device="cpu", pin_memory=True)
        h.copy_(t, non_blocking=True)
        return h

    def conv3x3_f32(self, dir, act, other, C, *a, **k):
        t = self._real.conv3x3_f32(dir, act, other, C, *a, **k)
        if VARIANT == "pinned" and dir == 1 and tuple(act.shape) == SHAPE:
            # the data gradient that feeds layer3.0's output: inputs + output, device-allocation free
            self._log.append(("dgrad", {"dy": self._pin(act), "w": self._pin(other), "dx": self._pin(C),
                                        "dx_ptr": C.data_ptr(), "args": [repr(v) for v in a]}))
        return t

    def bn_act_fwd(self, x, res, *a):
        out = self._real.bn_act_fwd(x, res, *a)
        if VARIANT == "pinned" and tuple(x.shape) == SHAPE and res is not None:
            self._log.append(("fwd", {"x": self._pin(x), "y": self._pin(out[0]), "save": self._pin(out[1]),
                                      "mask": self._pin(out[2]), "save_ptr": out[1].data_ptr()}))
            return out
        if tuple(x.shape) == SHAPE and res is not None:
            torch.cuda.synchronize()
            self._log.append(("fwd", {"x": x.clone(), "res": res.clone(), "y": out[0].clone(), "save": out[1].clone(),
                                      "mask": out[2].clone() if out[2] is not None and out[2].numel() else None,
                                      "save_ptr": out[1].data_ptr(), "x_ptr": x.data_ptr()}))
        return out

    def bn_act_fwd_partials(self, x, res, *a):
        out = self._real.bn_act_fwd_partials(x, res, *a)
        if VARIANT == "pinned" and tuple(x.shape) == SHAPE and res is not None:
            self._log.append(("fwd", {"x": self._pin(x), "y": self._pin(out[0]), "save": self._pin(out[1]),
                                      "mask": self._pin(out[2]), "save_ptr": out[1].data_ptr()}))
            return out
        if tuple(x.shape) == SHAPE and res is not None:
            torch.cuda.synchronize()
            self._log.append(("fwd", {"x": x.clone(), "res": res.clone(), "y": out[0].clone(), "save": out[1].clone(),
                                      "mask": out[2].clone() if out[2] is not None and out[2].numel() else None,
                                      "save_ptr": out[1].data_ptr(), "x_ptr": x.data_ptr()}))
        return out

    def bn_act_bwd(self, dy, dy2, x, mask, weight, save, relu, want_dres, want_w, det, tw, tb):
        pre = None
        hit = tuple(x.shape) == SHAPE and dy2 is not None
        if hit and VARIANT == "pinned":
            pre = {"dy": self._pin(dy), "dy2": self._pin(dy2), "x": self._pin(x), "mask": self._pin(mask),
                   "save": self._pin(save), "weight": self._pin(weight), "save_ptr": save.data_ptr()}
            out = self._real.bn_act_bwd(dy, dy2, x, mask, weight, save, relu, want_dres, want_w, det, tw, tb)
            pre.update({"dx": self._pin(out[0]), "dres": self._pin(out[1]), "dw": self._pin(out[2]),
                        "db": self._pin(out[3]), "relu": relu, "dy_post": self._pin(dy), "dy2_post": self._pin(dy2)})
            self._log.append(("bwd", pre))
            return out
        if hit and VARIANT in ("sync_after", "keep", "dummy_before"):
            if VARIANT == "dummy_before":
                dy.add_(0.0)  # one trivial kernel on the same stream between producer and BN
            out = self._real.bn_act_bwd(dy, dy2, x, mask, weight, save, relu, want_dres, want_w, det, tw, tb)
            if VARIANT == "sync_after":
                torch.cuda.synchronize()
            if VARIANT == "keep":  # references only: checked after backward, no sync here
                self.kept.append({"dy": dy, "dy2": dy2, "x": x, "mask": mask, "save": save, "weight": weight,
                                  "dx": out[0], "dres": out[1], "dw": out[2], "db": out[3]})
            return out
        if hit and VARIANT == "sync_before":
            torch.cuda.synchronize()
            return self._real.bn_act_bwd(dy, dy2, x, mask, weight, save, relu, want_dres, want_w, det, tw, tb)
        if hit:
            torch.cuda.synchronize()
            pre = {"dy": dy.clone(), "dy2": dy2.clone(), "x": x.clone(), "mask": mask.clone() if mask is not None else None,
                   "save": save.clone(), "weight": weight.clone(), "save_ptr": save.data_ptr(), "x_ptr": x.data_ptr()}
        out = self._real.bn_act_bwd(dy, dy2, x, mask, weight, save, relu, want_dres, want_w, det, tw, tb)
        if pre is not None:
            torch.cuda.synchronize()
            pre.update({"dx": out[0].clone(), "dres": out[1].clone() if out[1] is not None else None,
                        "dw": out[2].clone(), "db": out[3].clone(), "relu": relu,
                        "dy_post": dy.clone(), "dy2_post": dy2.clone()})
            self._log.append(("bwd", pre))
        return out


def unpack_mask(mask, M, C):
    bits = torch.stack([(mask >> j) & 1 for j in range(8)], dim=1).reshape(-1)[: M * C]
    return bits.reshape(M, C).bool()


def ref_bwd(b):
    """fp64 BN(+residual)+ReLU backward from the captured inputs (rows = N*H*W, channels_last)."""
    M, C = SHAPE[0] * SHAPE[2] * SHAPE[3], SHAPE[1]
    rows = lambda t: t.permute(0, 2, 3, 1).reshape(M, C).double().cpu()  # noqa: E731
    x, dy, dy2 = rows(b["x"]), rows(b["dy"]), rows(b["dy2"])
    mean, invstd = b["save"][:C].double().cpu(), b["save"][C:2 * C].double().cpu()
    g = b["weight"].double().cpu()
    m = unpack_mask(b["mask"].cpu(), M, C) if b["mask"] is not None else torch.ones(M, C, dtype=torch.bool)
    dz = (dy + dy2) * m
    xh = (x - mean) * invstd
    db = dz.sum(0)
    dw = (dz * xh).sum(0)
    dx = g * invstd / M * (M * dz - db - xh * dw)
    return dx, dz, dw, db, rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", default="dgrad=mfma_t2")
    ap.add_argument("--modes", default="ddp_off,ddp_on")
    ap.add_argument("--variant", default="sync_both")
    args = ap.parse_args()
    global VARIANT
    VARIANT = args.variant
    forced = dict(kv.split("=") for kv in args.force.split(",") if kv)
    pick3, pick_bn = conv._pick3, conv._pick_bn
    conv._pick3 = lambda d, x, w, dy, s: (forced[d] if d in forced and not (d == "dgrad" and (s != 1 or w.shape[2] != 3))
                                          else pick3(d, x, w, dy, s))
    conv._pick_bn = lambda cv, bn, x, r, relu: forced.get("bn") or pick_bn(cv, bn, x, r, relu)

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(D._port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    log = []
    proxy = Proxy(_native.lib(), log)
    _native._lib = proxy

    torch.manual_seed(0)
    base = D.resnet18_cifar()
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8, 3, 16, 16, generator=g)
    y = torch.randint(0, 10, (8,), generator=g)
    ref_model = copy.deepcopy(base).double()
    ref_act = {}
    for nm in ("layer3.0", "layer3.1"):  # fp64 forward outputs (the block output's ReLU pattern)
        dict(ref_model.named_modules())[nm].register_forward_hook(
            lambda mod, i, o, nm=nm: ref_act.__setitem__(nm, (o[0] if isinstance(o, tuple) else o).detach().clone()))
    _, ref_g, ref_m = D.run(ref_model, x.double(), y, torch.device("cpu"), False, False)
    for mode in args.modes.split(","):
        log.clear()
        proxy.kept.clear()
        _, gr, _ = D.run(base, x, y, torch.device("cuda", 0), ddp=mode.startswith("ddp"), stream_on="_on" in mode)
        torch.cuda.synchronize()
        perr = D.rel(gr["layer3.0.bn2.bias"], ref_g["layer3.0.bn2.bias"])
        fw = [d for k, d in log if k == "fwd"]
        bw = [d for k, d in log if k == "bwd"]
        rep = {"mode": mode, "force": args.force, "variant": args.variant, "bn2_bias_rel_err": perr,
               "n_fwd": len(fw), "n_bwd": len(bw)}
        for i, k in enumerate(proxy.kept):  # outputs vs an fp64 recomputation from the kernel's own inputs
            kk = {n: (v.clone() if isinstance(v, torch.Tensor) else v) for n, v in k.items()}
            dx, dz, dw, db, rows = ref_bwd(kk)
            rep[f"kept{i}"] = {"dx_rel": D.rel(rows(kk["dx"]), dx), "db_rel": D.rel(kk["db"].double().cpu(), db),
                               "dw_rel": D.rel(kk["dw"].double().cpu(), dw),
                               "dres_rel": None if kk["dres"] is None else D.rel(rows(kk["dres"]), dz)}
        for i, dg in enumerate([d for k, d in log if k == "dgrad"]):
            ref = torch.nn.grad.conv2d_input((8, 256, 4, 4), dg["w"].double(), dg["dy"].double(), padding=1)
            rep[f"dgrad{i}"] = {"rel": D.rel(dg["dx"].double(), ref), "args": dg["args"]}
        for i, b in enumerate(bw):
            f = [d for d in fw if d["save_ptr"] == b["save_ptr"]]
            f = f[-1] if f else None
            dx, dz, dw, db, rows = ref_bwd(b)
            r = {"x_same_as_fwd": None if f is None else bool(torch.equal(f["x"], b["x"])),
                 "save_same_as_fwd": None if f is None else bool(torch.equal(f["save"], b["save"])),
                 "mask_same_as_fwd": None if f is None or f["mask"] is None else bool(torch.equal(f["mask"], b["mask"])),
                 "dy_changed_during_kernel": not torch.equal(b["dy"], b["dy_post"]),
                 "dy2_changed_during_kernel": not torch.equal(b["dy2"], b["dy2_post"]),
                 "dx_rel": D.rel(rows(b["dx"]), dx), "db_rel": D.rel(b["db"].double().cpu(), db),
                 "dw_rel": D.rel(b["dw"].double().cpu(), dw),
                 "dres_rel": None if b["dres"] is None else D.rel(rows(b["dres"]), dz)}
            if f is not None and f["mask"] is not None:
                # the mask the forward should have written: y > 0
                yr = f["y"].permute(0, 2, 3, 1).reshape(-1, SHAPE[1]).cpu() > 0
                r["fwd_mask_matches_y"] = bool(torch.equal(unpack_mask(f["mask"].cpu(), *yr.shape), yr))
            # which layer / is the kernel's dbias what ends up in .grad / were its input gradients right
            r["db_vs_grad"] = {n: D.rel(b["db"].double().cpu(), gr[n]) for n in ("layer3.0.bn2.bias", "layer3.1.bn2.bias")}
            r["db_vs_fp64"] = {n: D.rel(b["db"].double().cpu(), ref_g[n]) for n in ("layer3.0.bn2.bias", "layer3.1.bn2.bias")}
            dsum = (b["dy"].double() + b["dy2"].double()).cpu()
            r["dy_sum_vs_fp64"] = {k: D.rel(dsum, ref_m[k]) for k in ("layer3.0[full]", "layer3.1[full]") if k in ref_m}
            m_cap = unpack_mask(b["mask"].cpu(), 128, 256)
            for nm, ya in ref_act.items():
                yr = ya.permute(0, 2, 3, 1).reshape(128, 256) > 0
                r[f"mask_vs_fp64_{nm}"] = int((m_cap != yr).sum())  # disagreeing ReLU bits
            if f is not None:
                yg = f["y"].permute(0, 2, 3, 1).reshape(128, 256).double()
                r["fwd_y_vs_fp64"] = {nm: D.rel(yg, ya.permute(0, 2, 3, 1).reshape(128, 256)) for nm, ya in ref_act.items()}
            rep[f"bwd{i}"] = r
        print(json.dumps(rep), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
