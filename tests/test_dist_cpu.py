"""World-size-2 gloo tests of the data-parallel path (qdiff.dist, bench.py's N>1 step) on CPU.

The N>1 bench shards prompts across ranks with no per-step collective: rank 0 broadcasts the
full CFG text-embedding batch, every rank denoises its own shard, latents are gathered to rank 0
and the timed region is max-reduced over ranks.  These tests run the exact
qdiff.dist functions bench.py calls, over gloo, in two spawned processes (127.0.0.1 rendezvous).
"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        import qdiff_boot  # noqa: F401
        from qdiff import dist as qdist
        r, w, local = qdist.init_from_env(backend="gloo")
        assert (r, w, local) == (rank, world, rank)
        B = 3  # prompts per rank
        # rank 0 owns the real context; others start from garbage and receive the broadcast
        full = torch.arange(2 * B * world * 5 * 4, dtype=torch.float32).view(2 * B * world, 5, 4)
        ctx = full.clone() if rank == 0 else torch.full_like(full, -1.0)
        qdist.broadcast_context(ctx, 0)
        assert torch.equal(ctx, full)
        mine = qdist.shard_context(ctx, rank, world)
        # uncond rows of this rank's prompts, then their cond rows
        s, e = qdist.shard_range(B * world, rank, world)
        assert torch.equal(mine[:B], full[s:e]) and torch.equal(mine[B:], full[B * world + s:B * world + e])
        # "denoise": a deterministic per-rank function of the shard
        lat = mine[:B, :1, :].clone() * 2 + rank
        out = qdist.gather_latents(lat, 0)
        if rank == 0:
            ref = torch.cat([full[a * B:(a + 1) * B, :1, :] * 2 + a for a in range(world)])
            assert torch.equal(out, ref)
        else:
            assert out is None
        # GEMM table sharing (bench.py before warm-up): rank 0 tunes, every rank ends with its table
        from qdiff import kernels as K
        key = ("linear", 4096, 320, 320, 320, 1, 0, ("f16",))

        def warm():
            K._TUNE[key] = (0, 103)

        shared = qdist.share_gemm_table(warm, rank, world)
        assert K._TUNE.get(key) == (0, 103) and [list(key[:7]) + [["f16"]], [0, 103]] in shared
        # bench.py timing reduction: MAX over ranks
        t = torch.tensor([1.0 + rank], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        assert t.item() == float(world)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


def test_shard_range_covers_everything():
    sys.path.insert(0, ROOT)
    import qdiff_boot  # noqa: F401
    from qdiff import dist as qdist
    for total in (0, 1, 7, 8, 16):
        for world in (1, 2, 3, 8):
            spans = [qdist.shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.timeout(120)
def test_gloo_world2_broadcast_shard_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=110) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    assert res == {0: "ok", 1: "ok"}, res


def test_table_export_import_roundtrip(tmp_path):
    sys.path.insert(0, ROOT)
    import json
    import qdiff_boot  # noqa: F401
    from qdiff import kernels as K
    saved = dict(K._TUNE)
    try:
        K._TUNE.clear()
        K._TUNE[("conv", 8, 64, 64, 320, 320, 3, 3, 1, 1, False, 5)] = (0, 200)
        K._TUNE[("linear", 8, 1280, 320, 320, 1, 0, ("i8", "f16"))] = None
        blob = json.dumps(K.export_table())
        K._TUNE.clear()
        assert K.import_table(json.loads(blob)) == 2
        assert K._TUNE[("conv", 8, 64, 64, 320, 320, 3, 3, 1, 1, False, 5)] == (0, 200)
        assert K._TUNE[("linear", 8, 1280, 320, 320, 1, 0, ("i8", "f16"))] is None
    finally:
        K._TUNE.clear()
        K._TUNE.update(saved)


def test_bench_gpus_n_launches_n_ranks(monkeypatch):
    """`python bench.py --gpus N` outside torchrun starts N ranks through torch.distributed.run
    (127.0.0.1 rendezvous) from a parent that never touches the GPU, and returns their status."""
    import subprocess
    sys.path.insert(0, ROOT)
    import bench
    calls = []

    def fake_call(cmd, env=None):
        calls.append((cmd, env))
        return 3

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    with pytest.raises(SystemExit) as ei:
        bench.main()
    assert ei.value.code == 3
    cmd, env = calls[0]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[-4:] == ["--gpus", "4", "--steps", "2"]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert not torch.cuda.is_initialized()
