"""TEST-ONLY communicator: GPU buffers staged through host memory and the gloo process group.

RCCL refuses two ranks of one communicator on the same GPU ("Using the same HIP device for multiple
ranks of the same Communicator is not supported", rccl.h:174-176), and the GPU box has one GPU.  To
exercise the engine's multi-rank orchestration (Layout R buckets, in-place reduce-scatter /
all-gather slices, ZeRO-1 carry, per-rank Adam windows) with the real HIP pack / Adam / unpack
kernels, ws processes share cuda:0 and exchange through this class.  Sums are done in fp32.
"""
import torch
import torch.distributed as dist


class GlooStagedComm:
    def __init__(self, group=None):
        self.group = group
        self.ws = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.calls = []

    def reduce_scatter(self, send, recv, stream):
        stream.synchronize()
        h = send.detach().to("cpu", torch.float32)
        out = torch.empty(recv.numel(), dtype=torch.float32)
        dist.reduce_scatter_tensor(out, h, group=self.group)
        with torch.cuda.stream(stream):
            recv.copy_(out.to(recv.device).to(recv.dtype))
        self.calls.append(("rs", send.numel()))

    def all_gather(self, send, recv, stream):
        stream.synchronize()
        h = send.detach().to("cpu")
        if h.dtype != torch.float32:  # a gather is a byte copy: move bf16 / uint8 as int8 bytes
            h = h.view(torch.int8)
        out = torch.empty(recv.numel() * recv.element_size() // h.element_size(), dtype=h.dtype)
        dist.all_gather_into_tensor(out, h, group=self.group)
        out = out.view(recv.dtype)
        with torch.cuda.stream(stream):
            recv.copy_(out.to(recv.device))
        self.calls.append(("ag", recv.numel()))

    def _root(self, root):
        return dist.get_global_rank(self.group, root) if self.group else root

    def reduce(self, t, root, stream):
        stream.synchronize()
        h = t.detach().to("cpu", torch.float32)
        dist.reduce(h, dst=self._root(root), group=self.group)
        if root == self.rank:
            with torch.cuda.stream(stream):
                t.copy_(h.to(t.device).to(t.dtype))
        self.calls.append(("reduce", t.numel()))

    def broadcast(self, t, root, stream):
        stream.synchronize()
        h = t.detach().to("cpu")
        if h.dtype != torch.float32:
            h = h.view(torch.int8)
        dist.broadcast(h, src=self._root(root), group=self.group)
        h = h.view(t.dtype)
        with torch.cuda.stream(stream):
            t.copy_(h.to(t.device))
        self.calls.append(("bcast", t.numel()))

    def reduce_v(self, buf, win_off, win_len, stream):
        stream.synchronize()
        h = buf.detach().to("cpu", torch.float32)
        for root, (off, n) in enumerate(zip(win_off, win_len)):
            if n:
                part = h[int(off):int(off) + int(n)].clone()
                dist.reduce(part, dst=dist.get_global_rank(self.group, root) if self.group else root,
                            group=self.group)
                if root == self.rank:
                    h[int(off):int(off) + int(n)] = part
        with torch.cuda.stream(stream):
            buf.copy_(h.to(buf.device).to(buf.dtype))
        self.calls.append(("rsv", int(sum(win_len))))

    def broadcast_v(self, buf, win_off, win_len, stream):
        stream.synchronize()
        h = buf.detach().to("cpu")
        for root, (off, n) in enumerate(zip(win_off, win_len)):
            if n:
                part = h[int(off):int(off) + int(n)].clone()
                raw = part if part.dtype == torch.float32 else part.view(torch.int8)
                dist.broadcast(raw, src=self._root(root), group=self.group)
                h[int(off):int(off) + int(n)] = raw.view(part.dtype)
        with torch.cuda.stream(stream):
            buf.copy_(h.to(buf.device))
        self.calls.append(("agv", int(sum(win_len))))

    def all_reduce(self, t, stream):
        stream.synchronize()
        h = t.detach().to("cpu", torch.float32)
        dist.all_reduce(h, group=self.group)
        with torch.cuda.stream(stream):
            t.copy_(h.to(t.device).to(t.dtype))
        self.calls.append(("ar", t.numel()))
