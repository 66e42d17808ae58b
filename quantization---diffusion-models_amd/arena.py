"""Static activation arena for the captured denoising step.

The UNet step is a fixed sequence of kernel launches over fixed shapes, so every intermediate
buffer can be planned once: the warm-up step records the allocation sequence (shape, dtype)
and allocates each buffer persistently; every later step - in particular the hipGraph capture
and all replays - receives exactly the same buffers in the same order.  Nothing is allocated
while a graph is being captured, and the graph only ever references memory the loop owns, so
no interaction with the caching allocator's pools can alias a live graph buffer.

With 288 GB of HBM per MI355X the plan keeps every intermediate of one step resident (SD1.5,
UNet batch 8 at 64x64 latents: a few GB) instead of recycling them.
"""
from contextlib import contextmanager

import torch

_active = None


class Arena:
    def __init__(self):
        self.bufs = []
        self.i = 0
        self.frozen = False
        # fp32 atomic-max targets that must start each step at zero: recorded individually on the
        # first step, then carved out of ONE pool that a single kernel zeroes at every step start
        self.zsizes = []
        self.zviews = None
        self.zpool = None
        self.zi = 0
        self.stream = None

    def zeroed_f32(self, n, device):
        """A zero-filled fp32 buffer of n elements for this step -> (tensor, True)."""
        self._check_stream(device)
        if self.zviews is not None:
            if self.zi >= len(self.zviews) or self.zviews[self.zi].numel() != n:
                raise RuntimeError(f"arena: zeroed buffer #{self.zi} changed size; the step is not shape-static")
            t = self.zviews[self.zi]
        else:
            if self.frozen:
                raise RuntimeError("arena: zeroed allocation beyond the recorded plan while frozen")
            self.zsizes.append(n)
            self.zdevice = device
            t = torch.zeros(n, dtype=torch.float32, device=device)
        self.zi += 1
        return t, True

    def _build_pool(self, device):
        tot = sum((n + 63) // 64 * 64 for n in self.zsizes)  # 256-B aligned slices
        self.zpool = torch.zeros(max(tot, 1), dtype=torch.float32, device=device)
        self.zviews, off = [], 0
        for n in self.zsizes:
            self.zviews.append(self.zpool[off:off + n])
            off += (n + 63) // 64 * 64

    def _check_stream(self, device):
        """The plan is one stream's launch order: every buffer is handed out assuming the launches
        that use it are ordered on that stream (the zero pool is cleared at the step start on it).
        A launch on another stream would race with that order, so a second stream is refused."""
        device = torch.device(device)
        if device.type != "cuda":
            return
        cur = torch.cuda.current_stream(device)
        if self.stream is None:
            self.stream = cur  # the step's stream (a graph capture runs on its own stream)
        elif cur != self.stream:
            raise RuntimeError("arena: buffers requested on a second stream; the step plan is single-stream")

    def begin_step(self):
        """Zero the pool (one launch, captured into the step's graph)."""
        self.i = 0
        self.zi = 0
        self.stream = None
        if self.zpool is not None:
            from . import _lib
            _lib.call("qd_fill_zero", self.zpool.data_ptr(), self.zpool.numel(),
                      torch.cuda.current_stream(self.zpool.device).cuda_stream)

    def end_step(self):
        if self.zviews is None and self.zsizes and not self.frozen:
            self._build_pool(self.zdevice)

    def alloc(self, shape, dtype, device):
        shape = torch.Size(shape)
        self._check_stream(device)
        if self.i < len(self.bufs):
            t = self.bufs[self.i]
            if t.shape != shape or t.dtype != dtype:
                raise RuntimeError(f"arena: allocation #{self.i} changed from {tuple(t.shape)}/{t.dtype} to "
                                   f"{tuple(shape)}/{dtype}; the step is not shape-static")
        else:
            if self.frozen:
                raise RuntimeError("arena: allocation beyond the recorded plan while frozen (graph capture)")
            t = torch.empty(shape, dtype=dtype, device=device)
            self.bufs.append(t)
        self.i += 1
        return t

    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in self.bufs)


@contextmanager
def using(arena, frozen=False):
    """Route kernels.empty() through `arena` for the duration of one step."""
    global _active
    prev = _active
    _active = arena
    arena.frozen = frozen
    arena.begin_step()
    try:
        yield arena
    finally:
        _active = prev
        arena.end_step()
        arena.frozen = False


def empty(shape, dtype, device):
    if _active is not None:
        return _active.alloc(shape, dtype, device)
    return torch.empty(shape, dtype=dtype, device=device)


def zeroed_f32(n, device):
    """(buffer, zeroed): inside an arena step a pooled zero-filled buffer (the consuming kernel
    may skip its own zero-fill); otherwise an uninitialised one the kernel must zero itself."""
    if _active is not None:
        return _active.zeroed_f32(n, device)
    return torch.empty(n, dtype=torch.float32, device=device), False
