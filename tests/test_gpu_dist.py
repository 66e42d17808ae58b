"""Multi-rank denoising on the GPU box: two ranks (gloo, both on the box's one
GPU) run the product's data-parallel path - rank 0 tunes and broadcasts the GEMM table, rank 0
broadcasts the CFG text context, each rank denoises its prompt shard with the graph-replayed
DenoiseLoop, latents are gathered to rank 0 - and the gathered latents must equal, bit for bit,
one process running the same shards one after the other with the same kernel table."""
import json
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

PROMPTS, WORLD, STEPS = 4, 2, 3


def _setup(seed=7):
    from qdiff.models import StableDiffusion1_x
    model = StableDiffusion1_x.from_pretrained("synthetic:tiny", device="cuda:0", seed=seed)
    model.quantize(quant_config=dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True), quantUnet=True)
    cfg = model.pipeline.unet.config
    g = torch.Generator().manual_seed(42)
    lat = torch.randn(PROMPTS, 4, cfg.sample_size, cfg.sample_size, generator=g).half()
    ctx = torch.randn(2 * PROMPTS, 77, cfg.cross_attention_dim, generator=g).half()
    return model, cfg, lat, ctx


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, port, out_dir):
    import sys
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import qdiff_boot  # noqa: F401  (registers the package as `qdiff` in the spawned process)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK="0")
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    torch.cuda.set_device(0)
    from qdiff import dist as qdist
    model, cfg, lat, ctx = _setup()
    dev = torch.device("cuda:0")
    b = PROMPTS // WORLD
    loop = model.get_loop(b, cfg.sample_size * 8, cfg.sample_size * 8, STEPS, 7.5)
    full = ctx.to(dev) if rank == 0 else torch.zeros_like(ctx, device=dev)
    lat_r = lat[rank * b:(rank + 1) * b]

    def warm():
        loop.set_inputs(lat_r, qdist.shard_context(full, rank, WORLD))
        loop.step()

    table = qdist.share_gemm_table(warm, rank, WORLD)
    qdist.broadcast_context(full, 0)
    out = loop.run(lat_r, qdist.shard_context(full, rank, WORLD))
    got = qdist.gather_latents(out, 0)
    if rank == 0:
        torch.save(got.cpu(), os.path.join(out_dir, "gathered.pt"))
        with open(os.path.join(out_dir, "table.json"), "w") as f:
            json.dump(table, f)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_denoise_equals_sequential_shards(tmp_path):
    import torch.multiprocessing as mp
    from qdiff import dist as qdist
    from qdiff import kernels as K
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_worker, args=(port, str(tmp_path)), nprocs=WORLD, start_method="spawn", join=True)
    gathered = torch.load(tmp_path / "gathered.pt", weights_only=True)
    with open(tmp_path / "table.json") as f:
        K.import_table(json.load(f))
    model, cfg, lat, ctx = _setup()
    dev = torch.device("cuda:0")
    b = PROMPTS // WORLD
    loop = model.get_loop(b, cfg.sample_size * 8, cfg.sample_size * 8, STEPS, 7.5)
    outs = [loop.run(lat[r * b:(r + 1) * b], qdist.shard_context(ctx.to(dev), r, WORLD)).cpu() for r in range(WORLD)]
    ref = torch.cat(outs)
    print("sharded vs sequential max |diff|", (gathered.float() - ref.float()).abs().max().item())
    assert gathered.shape == (PROMPTS, 4, cfg.sample_size, cfg.sample_size)
    assert torch.isfinite(gathered.float()).all()
    assert torch.equal(gathered, ref)
