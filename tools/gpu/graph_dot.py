"""Capture a bench workload's whole-step HIP graph with the debug dump on and report its shape:
nodes, roots, LEAVES (nodes nothing depends on) and the kernels on them.  A leaf other than the
step's last node is a branch the graph launch does not join -- the next replay may overlap it.
Usage: python tools/gpu/graph_dot.py --workload bert_none [--out gpurun_out/bert.dot]
"""
import argparse
import collections
import os
import re
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from grace_amd import grace_from_params  # noqa: E402
from grace_amd.parallel import DistributedOptimizer, FusedSGD  # noqa: E402
from grace_amd.utils.workloads import WORKLOADS, build_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="bert_none")
    ap.add_argument("--out", default="gpurun_out/graph.dot")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    torch.manual_seed(0)
    model = build_model(w, dev)
    named = list(model.named_parameters())
    opt = DistributedOptimizer(FusedSGD([p for _, p in named], lr=0.01, momentum=0.5),
                               grace_from_params(dict(w.grace, world_size=1)), named_parameters=named,
                               bucket_cap_mb=128.0, overlap=False)
    data = w.make_batch(w.batch, dev)
    if w.channels_last:
        data = (data[0].contiguous(memory_format=torch.channels_last),) + tuple(data[1:])

    def step():
        opt.zero_grad(set_to_none=True)
        loss = w.loss(model, data)
        loss.backward()
        opt.step()
        return loss

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    try:
        g = torch.cuda.CUDAGraph(keep_graph=True)  # the raw hipGraph_t stays inspectable
    except TypeError:
        g = torch.cuda.CUDAGraph()
    g.enable_debug_mode()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    out = os.path.abspath(args.out)
    try:
        g.debug_dump(out)
    except Exception as e:  # noqa: BLE001
        print("debug_dump failed:", e)
    if not os.path.exists(out):
        return hip_walk(g, args.workload)
    text = open(out).read()
    # DOT: node lines  "name" [ ... label="..." ]  and edges  "a" -> "b"
    edges = re.findall(r'"?([\w.]+)"?\s*->\s*"?([\w.]+)"?', text)
    labels = {}
    for m in re.finditer(r'"?([\w.]+)"?\s*\[(.*?)\];?\s*$', text, re.M):
        lab = re.search(r'label="(.*?)"', m.group(2), re.S)
        labels[m.group(1)] = (lab.group(1) if lab else m.group(2))[:160].replace("\\n", " ")
    nodes = set(labels) | {a for a, _ in edges} | {b for _, b in edges}
    outd = collections.Counter(a for a, _ in edges)
    ind = collections.Counter(b for _, b in edges)
    leaves = [n for n in nodes if outd[n] == 0]
    roots = [n for n in nodes if ind[n] == 0]
    print(f"{args.workload}: {len(nodes)} nodes, {len(edges)} edges, {len(roots)} roots, {len(leaves)} leaves")
    for n in leaves[:20]:
        print("  leaf:", n, labels.get(n, "")[:200])
    for n in roots[:10]:
        print("  root:", n, labels.get(n, "")[:200])


def hip_walk(g, name):
    """The same census through the HIP graph API (ctypes on the process's libamdhip64)."""
    import ctypes

    raw = g.raw_cuda_graph() if hasattr(g, "raw_cuda_graph") else None
    if raw is None:
        print("no debug dump and no raw_cuda_graph(): cannot walk the graph")
        return
    hip = None
    for lib in ("libamdhip64.so", "libamdhip64.so.7"):
        try:
            hip = ctypes.CDLL(lib)
            break
        except OSError:
            continue
    graph = ctypes.c_void_p(raw)
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(graph, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(graph, nodes, ctypes.byref(n)) == 0
    hip.hipKernelNameRefByPtr.restype = ctypes.c_char_p

    class KP(ctypes.Structure):  # hipKernelNodeParams
        _fields_ = [("blockDim", ctypes.c_uint * 3), ("extra", ctypes.c_void_p), ("func", ctypes.c_void_p),
                    ("gridDim", ctypes.c_uint * 3), ("kernelParams", ctypes.c_void_p), ("sharedMemBytes", ctypes.c_uint)]

    def label(nd):
        t = ctypes.c_int(0)
        hip.hipGraphNodeGetType(nd, ctypes.byref(t))
        if t.value == 0:  # kernel
            kp = KP()
            if hip.hipGraphKernelNodeGetParams(nd, ctypes.byref(kp)) == 0 and kp.func:
                nm = hip.hipKernelNameRefByPtr(ctypes.c_void_p(kp.func), None)
                return "kernel " + (nm.decode()[:120] if nm else hex(kp.func))
            return "kernel"
        return f"type {t.value}"

    leaves, roots, deg = [], [], {}
    for i in range(n.value):
        nd = ctypes.c_void_p(nodes[i])
        k = ctypes.c_size_t(0)
        hip.hipGraphNodeGetDependentNodes(nd, None, ctypes.byref(k))
        d = ctypes.c_size_t(0)
        hip.hipGraphNodeGetDependencies(nd, None, ctypes.byref(d))
        deg[i] = (d.value, k.value)
        if k.value == 0:
            leaves.append(i)
        if d.value == 0:
            roots.append(i)
    print(f"{name}: {n.value} nodes, {len(roots)} roots, {len(leaves)} leaves (hip walk)")
    for i in leaves[:20]:
        print("  leaf:", i, label(ctypes.c_void_p(nodes[i])))
    for i in roots[:10]:
        print("  root:", i, label(ctypes.c_void_p(nodes[i])))
    fan = sorted(((v[1], i) for i, v in deg.items()), reverse=True)[:5]
    print("  max fan-out:", [(f, label(ctypes.c_void_p(nodes[i]))) for f, i in fan])


if __name__ == "__main__":
    main()
