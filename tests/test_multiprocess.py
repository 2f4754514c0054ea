"""World-size-2 gloo tests of the multi-GPU plumbing (file-parallel sharding, max-over-ranks timing),
run on CPU with the oracle standing in for the per-rank work."""
import os
import socket

import pytest
import torch.multiprocessing as mp

import shard


def test_shard_files_lpt():
    sizes = [128, 64, 64, 32, 32, 32, 16, 8, 8, 1]
    sh = shard.shard_files(sizes, 3)
    assert sorted(i for s in sh for i in s) == list(range(len(sizes)))
    loads = [sum(sizes[i] for i in s) for s in sh]
    assert max(loads) - min(loads) <= 16
    # config 4 shape: 1024 equal files over 8 GPUs -> 128 each
    sh8 = shard.shard_files([128 << 20] * 1024, 8)
    assert [len(s) for s in sh8] == [128] * 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import oracle_ctypes as O
    dist = shard.init_distributed("gloo")
    seed = bytes([1, 2, 3, 4])
    sizes = [3000 + 517 * i for i in range(9)]
    mine = shard.shard_files(sizes, world)[rank]
    lit = mat = 0
    for i in mine:
        basis = O.splitmix(sizes[i], 1000 + i)
        src = basis.copy()
        src[100:900] = O.splitmix(800, 2000 + i)
        h = O.header(512, 2, basis.size)
        w, s = O.generator(basis, h, seed)
        _, _, l, m, _ = O.sender(src, h, w, s, seed)
        lit += l
        mat += m
    tot_lit = shard.reduce_over_ranks(lit, "sum")
    tot_mat = shard.reduce_over_ranks(mat, "sum")
    tmax = shard.reduce_over_ranks(float(rank + 1), "max")
    out[rank] = (tot_lit, tot_mat, tmax, len(mine))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_file_sharding():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    import oracle_ctypes as O
    seed = bytes([1, 2, 3, 4])
    sizes = [3000 + 517 * i for i in range(9)]
    lit = mat = 0
    for i in range(len(sizes)):
        basis = O.splitmix(sizes[i], 1000 + i)
        src = basis.copy()
        src[100:900] = O.splitmix(800, 2000 + i)
        h = O.header(512, 2, basis.size)
        w, s = O.generator(basis, h, seed)
        _, _, l, m, _ = O.sender(src, h, w, s, seed)
        lit += l
        mat += m
    assert out[0][:3] == out[1][:3] == (lit, mat, 2.0)
    assert out[0][3] + out[1][3] == len(sizes)


def test_bench_gpus2_dry_run_spawns_ranks():
    """`python bench.py --gpus 2` without a launcher starts the two rank processes itself (bench.spawn_ranks);
    --dry-run keeps them off the device (gloo).  The line must come from rank 0 and report both ranks, with
    the 256-file list (128 per GPU) sharded over them."""
    import json
    import subprocess
    import sys
    from conftest import ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                          "--workload", "files"], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["dry_run"] and rec["config"]["files_total"] == 256


def test_bench_gpus8_dry_run_reports_config4_list():
    """The driver's 8-GPU line (`python bench.py --gpus 8`, default workload) carries BASELINE config 4's files
    block: the 1024-file list sharded 128 per rank over a process group of 8 (gloo here, RCCL on the node)."""
    import json
    import subprocess
    import sys
    from conftest import ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--dry-run"],
                         capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8 and rec["files"]["files_total"] == 1024
    assert rec["files"]["files_per_gpu"] == 128 and rec["files"]["world_size_seen"] == 8


def test_rank_device_plan(monkeypatch):
    """One GPU per local rank: RCCL on the rank's own device.  More local ranks than GPUs (a rehearsal of the
    N-rank launch on a smaller box): round-robin devices and gloo, chosen identically by every rank."""
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert [shard.rank_device(r, 8, 8) for r in range(8)] == [(r, "nccl", False) for r in range(8)]
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert [shard.rank_device(r, 2, 1) for r in range(2)] == [(0, "gloo", True), (0, "gloo", True)]
    monkeypatch.delenv("LOCAL_WORLD_SIZE")
    assert [shard.rank_device(r, 4, 2) for r in range(4)] == [(0, "gloo", True), (1, "gloo", True),
                                                              (0, "gloo", True), (1, "gloo", True)]
    with pytest.raises(RuntimeError):
        shard.rank_device(0, 1, 0)


def test_bench_traffic_profiles_name_the_kernels():
    """bench.py's roofline.traffic comes from committed FETCH_SIZE passes (profiles/, rocprofv3 --pmc): the kernel names
    it looks for must be the ones those passes recorded, for both lines (a renamed instantiation once left the config-4
    line's traffic null)."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    n = 16 << 30
    for csv_rel, kernel in ((b.TRAFFIC_CSV, b.PROD_KERNEL), (b.TRAFFIC_FILES_CSV, b.BATCH_KERNEL)):
        t = b.pmc_traffic(os.path.join(root, "profiles", csv_rel), kernel, n)
        assert t is not None and 0.95 * n <= t <= 1.1 * n, (csv_rel, kernel, t)
