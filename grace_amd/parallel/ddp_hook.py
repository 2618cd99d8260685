"""GRACE as a ``torch.nn.parallel.DistributedDataParallel`` communication hook.

The reference predates DDP comm hooks (survey 2.12); this is the north-star integration:
``ddp.register_comm_hook(GraceHookState(grc), grace_comm_hook)`` and DDP's own bucketing,
backward overlap and gradient copy-back drive the GRACE pipeline.

For each DDP bucket the hook (called from the autograd thread as soon as the bucket is ready):
  1. registers the bucket's parameter layout (per-parameter compression semantics),
  2. forks a side **compress stream** from the compute stream and on it runs the fused
     compress kernels, the async RCCL collective and the one-pass decompress/aggregate,
  3. returns a ``torch.futures.Future`` completed on that side stream -- DDP's finaliser waits
     on its CUDA event, so backward compute is never blocked by the collective.
"""
from typing import Dict

import torch
import torch.distributed as dist

from ..core import Communicator, register_layout
from ..ops.layout import SegmentLayout


class GraceHookState:
    def __init__(self, grc: Communicator, name: str = "ddp"):
        self.grc = grc
        self.name = name
        self.layouts: Dict[int, SegmentLayout] = {}
        self.streams: Dict[int, torch.cuda.Stream] = {}

    def layout_for(self, bucket) -> str:
        idx = bucket.index()
        key = f"{self.name}.bucket{idx}"
        lay = self.layouts.get(idx)
        buf = bucket.buffer()
        if lay is None or lay.total != buf.numel():
            grads = bucket.gradients()
            lay = SegmentLayout.from_tensors(grads)
            if lay.total != buf.numel():  # padding inside the bucket: single segment
                lay = SegmentLayout((buf.numel(),), ((buf.numel(),),))
            self.layouts[idx] = lay
            register_layout(key, lay)
        return key


def grace_comm_hook(state: GraceHookState, bucket: dist.GradBucket) -> torch.futures.Future[torch.Tensor]:
    buf = bucket.buffer()
    name = state.layout_for(bucket)
    grc = state.grc
    if not buf.is_cuda:
        out = grc.step(buf if buf.dtype == torch.float32 else buf.float(), name)
        fut = torch.futures.Future()
        fut.set_result(out.to(buf.dtype).view_as(buf))
        return fut
    dev = buf.device
    s = state.streams.get(dev.index)
    if s is None:
        s = state.streams[dev.index] = torch.cuda.Stream(dev)
    cur = torch.cuda.current_stream(dev)
    s.wait_stream(cur)
    fut = torch.futures.Future(devices=[dev])
    with torch.cuda.stream(s):
        g = buf if buf.dtype == torch.float32 else buf.float()
        handles, ctx = grc.send_step(g, name)
        out = grc.receive_step(handles, ctx)
        out = out.to(buf.dtype).view_as(buf)
        buf.record_stream(s)
        fut.set_result(out)
    return fut
