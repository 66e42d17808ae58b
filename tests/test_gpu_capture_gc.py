"""Regression test for the round-5 capture abort: a dead Python reference
cycle that still owns HIP objects (an earlier denoising loop with its graph, an event, a stream) was
finalised by the garbage collector INSIDE a later loop's stream capture, and the destructors' HIP
calls, illegal while a stream captures, aborted the process (gpurun_out/r05x_tests.log:23).
`DenoiseLoop.capture` (pipeline.py) collects before the capture and keeps the collector off during it.

The test plants such a cycle, then forces a collection at the first launch inside the next capture
(what an automatic collection did in the round-5 run): with the pre-capture collect there is nothing
left to finalise and the captured loop replays to the eager result; without it the process aborts
(scripts/capture_gc_negative.py shows that in a child process, run once as the last step of a GPU call:
profiles/r06_capture_gc_negative.log)."""
import gc

import pytest
import torch

pytestmark = pytest.mark.gpu


class _Junk:
    pass


def _plant_dead_cycle(loop):
    j = _Junk()
    j.me = j                       # the cycle: only the collector frees it
    j.loop = loop                  # a captured loop: its torch.cuda.CUDAGraph, arena, streams
    j.event = torch.cuda.Event(enable_timing=True)
    j.event.record()
    j.stream = torch.cuda.Stream()
    j.graph = loop.graph


def scenario(dev, force_collect_in_capture=True):
    """Returns (eager latents, graph latents) of loop 2, built after loop 1 died in a cycle."""
    from qdiff import kernels as K
    from qdiff import pipeline as P
    from qdiff.models import StableDiffusion1_x
    model = StableDiffusion1_x.from_pretrained("synthetic:tiny", device=str(dev))
    model.quantize(quant_config=dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True), quantUnet=True)
    unet = model.pipeline.unet
    cfg = unet.config
    s = cfg.sample_size
    g = torch.Generator().manual_seed(11)
    lat = torch.randn(1, 4, s, s, generator=g).half().to(dev)
    ctx = torch.randn(2, 77, cfg.cross_attention_dim, generator=g).half().to(dev)

    def loop(use_graph):
        return P.DenoiseLoop(unet, 1, 8 * s, 8 * s, num_inference_steps=3, device=str(dev), use_graph=use_graph)

    l1 = loop(True)
    l1.run(lat, ctx)
    assert l1.graph is not None
    _plant_dead_cycle(l1)
    del l1

    orig = K.timestep_embedding

    def collect_in_capture(*a, **kw):
        if force_collect_in_capture and torch.cuda.is_current_stream_capturing():
            gc.collect()   # an automatic collection at this point in the round-5 run
        return orig(*a, **kw)

    K.timestep_embedding = collect_in_capture
    try:
        l2 = loop(True)
        got = l2.run(lat, ctx).cpu()
    finally:
        K.timestep_embedding = orig
    eager = loop(False).run(lat, ctx).cpu()
    return eager, got


def test_capture_after_dead_cycle_owning_hip_objects(dev):
    eager, got = scenario(dev)
    assert torch.isfinite(got.float()).all()
    assert torch.equal(eager, got)
