"""Data-parallel correctness on CPU (gloo, 2 ranks).

SURVEY §4: (a) replicas stay bit-identical across ranks after N updates, and (b) the all-reduced
update equals the single-process update over the concatenated batch (fp32 tolerance).  The
same code path runs over RCCL on GPUs (backend chosen by ``init_distributed``).
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp
import yaml

from tests.conftest import ROOT, cfg_path

ABILENE = cfg_path("networks", "abilene", "abilene-in4-rand-cap1-2.graphml")
B_PER_RANK = 6
WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg():
    cfg = yaml.safe_load(open(cfg_path("config", "agent", "sample_agent.yaml")))
    cfg["actor_hidden_layer_nodes"] = [32]
    cfg["critic_hidden_layer_nodes"] = [16]
    return cfg


def _learner(dist_info=None, seed=3, zero=None):
    from gsc_amd.agents import DDPGLearner
    from gsc_amd.coordsim.reader import load_topology
    from gsc_amd.models import GraphSet
    gs = GraphSet([load_topology(ABILENE)], 24, "cpu")
    return DDPGLearner(_cfg(), 3, 24 * 1 * 3 * 24, gs, 1, 3, "cpu", dist_info, amp_bf16=False, seed=seed,
                       zero=zero), gs


def _batches(n_updates):
    from gsc_amd.agents import Batch
    g = torch.Generator().manual_seed(11)
    out = []
    for _ in range(n_updates):
        B = B_PER_RANK * WORLD
        obs = torch.rand(B, 24, 3, generator=g)
        obs[:, 11:] = 0
        nxt = torch.rand(B, 24, 3, generator=g)
        nxt[:, 11:] = 0
        out.append(Batch(obs, torch.zeros(B, dtype=torch.int64), torch.rand(B, 1728, generator=g),
                         torch.rand(B, generator=g) - 0.5, nxt, (torch.rand(B, generator=g) < 0.2).float()))
    return out


def _worker(rank, port, out_dir, n_updates):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from gsc_amd.agents import Batch
    from gsc_amd.parallel.dist import init_distributed, shutdown
    info = init_distributed("cpu")
    # different init seeds per rank: the learner must broadcast rank 0's replicas
    learner, _ = _learner(info, seed=3 if rank == 0 else 99)
    for b in _batches(n_updates):
        sl = slice(rank * B_PER_RANK, (rank + 1) * B_PER_RANK)
        learner.update(Batch(*(t[sl] for t in b)))
    torch.save({"actor": learner.actor_flat.flat.clone(), "critic": learner.critic_flat.flat.clone(),
                "target_actor": learner.target_actor_flat.flat.clone()}, os.path.join(out_dir, f"r{rank}.pt"))
    shutdown()


def test_dp_allreduce_matches_single_process():
    n_updates = 3
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(_free_port(), d, n_updates), nprocs=WORLD, join=True, start_method="spawn")
        r = [torch.load(os.path.join(d, f"r{i}.pt"), weights_only=True) for i in range(WORLD)]
    for k in r[0]:
        assert torch.equal(r[0][k], r[1][k]), f"{k} differs across ranks"
    ref, _ = _learner(None, seed=3)
    for b in _batches(n_updates):
        ref.update(b)
    torch.testing.assert_close(r[0]["critic"], ref.critic_flat.flat, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(r[0]["actor"], ref.actor_flat.flat, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(r[0]["target_actor"], ref.target_actor_flat.flat, rtol=1e-5, atol=1e-6)


def _trainer_worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from gsc_amd.agents import BatchedTrainer, TrainerConfig
    from gsc_amd.parallel.dist import init_distributed, shutdown
    from gsc_amd.sim.batched import load_batched_from_paths
    info = init_distributed("cpu")
    cfg = _cfg()
    os.chdir(ROOT)
    sim = load_batched_from_paths([ABILENE], cfg_path("service_functions", "abc.yaml"),
                                  cfg_path("config", "simulator", "sample_config.yaml"), cfg, 4, device="cpu",
                                  seed=1000 + rank, host_threads=1)
    tr = BatchedTrainer(cfg, sim, TrainerConfig(num_envs=4, batch_size=16, learning_starts=2, seed=5 + rank,
                                                check_every=0), info)
    for _ in range(5):
        tr.step()
    m = tr.metrics()
    torch.save({"actor": tr.learner.actor_flat.flat.clone(), "critic": tr.learner.critic_flat.flat.clone(),
                "succ": torch.tensor(m["succ"]), "updates": torch.tensor(tr.learner.updates)},
               os.path.join(out_dir, f"t{rank}.pt"))
    shutdown()


def _zero_worker(rank, port, out_dir, n_updates):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from gsc_amd.agents import Batch
    from gsc_amd.parallel.dist import init_distributed, shutdown
    info = init_distributed("cpu")
    learner, _ = _learner(info, seed=3 if rank == 0 else 99, zero=True)
    assert learner.zero and learner.actor_opt.zero is not None
    assert learner.actor_opt.m.numel() * WORLD == learner.actor_flat.flat.numel()   # moments of 1/W only
    for b in _batches(n_updates):
        sl = slice(rank * B_PER_RANK, (rank + 1) * B_PER_RANK)
        learner.update(Batch(*(t[sl] for t in b)))
    opt = learner.actor_opt.state_dict()                       # collective: full-length moments
    out = {f"{net}.{n}": p.detach().clone() for net in ("actor", "critic", "target_actor")
           for n, p in getattr(learner, net).named_parameters()}
    out["actor_m"] = opt["m"][:learner.actor_flat.numel].clone()
    out["flat"] = learner.actor_flat.flat.clone()
    torch.save(out, os.path.join(out_dir, f"z{rank}.pt"))
    shutdown()


def test_dp_sharded_optimizer_matches_single_process():
    """ZeRO-1 (reduce-scatter -> Adam on the rank's 1/W shard -> all-gather; :mod:`gsc_amd.parallel.zero`):
    replicas stay bit-identical across ranks and equal the single-process update on the concatenated
    batch (fp32 tolerance); each rank holds Adam moments for 1/W of the parameters."""
    n_updates = 3
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_zero_worker, args=(_free_port(), d, n_updates), nprocs=WORLD, join=True,
                           start_method="spawn")
        r = [torch.load(os.path.join(d, f"z{i}.pt"), weights_only=True) for i in range(WORLD)]
    assert torch.equal(r[0]["flat"], r[1]["flat"])
    for k in r[0]:
        assert torch.equal(r[0][k], r[1][k]), f"{k} differs across ranks"
    ref, _ = _learner(None, seed=3)
    for b in _batches(n_updates):
        ref.update(b)
    for net in ("actor", "critic", "target_actor"):
        for n, p in getattr(ref, net).named_parameters():
            torch.testing.assert_close(r[0][f"{net}.{n}"], p.detach(), rtol=1e-5, atol=1e-6)
    from gsc_amd.ops.optim import FlatParams  # noqa: F401
    torch.testing.assert_close(r[0]["actor_m"].norm(), ref.actor_opt.m[:ref.actor_flat.numel].norm(), rtol=1e-5,
                               atol=1e-7)


def _zero_resume_worker(rank, port, out_dir, src):
    """ZeRO-1 at W=2: resume from ``src`` (a non-ZeRO, single-process checkpoint) when given, else train
    2 updates and write the (collective) checkpoint; then one more update from a fresh learner that
    loads it."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from gsc_amd.agents import Batch
    from gsc_amd.parallel.dist import init_distributed, shutdown
    info = init_distributed("cpu")
    bs = _batches(3)
    sl = slice(rank * B_PER_RANK, (rank + 1) * B_PER_RANK)
    if src:
        sd = torch.load(src, weights_only=True)
    else:
        learner, _ = _learner(info, seed=3, zero=True)
        for b in bs[:2]:
            learner.update(Batch(*(t[sl] for t in b)))
        sd = learner.state_dict()              # collective (moments all-gathered)
        if rank == 0:
            torch.save(sd, os.path.join(out_dir, "zero_sd.pt"))
    fresh, _ = _learner(info, seed=77, zero=True)
    fresh.load_state_dict(sd)
    fresh.update(Batch(*(t[sl] for t in bs[2])))
    torch.save({f"{net}.{n}": p.detach().clone() for net in ("actor", "critic", "target_actor")
                for n, p in getattr(fresh, net).named_parameters()}, os.path.join(out_dir, f"zr{rank}.pt"))
    shutdown()


def test_dp_resume_across_zero_and_world_size():
    """Checkpoints are layout-free (packed per parameter): a ZeRO W=2 checkpoint resumes in one process
    without ZeRO, and a single-process checkpoint resumes under ZeRO W=2 -- both equal to the uninterrupted
    single-process run (the flat layout's bucket padding depends on the world size)."""
    from gsc_amd.agents import Batch  # noqa: F401
    bs = _batches(3)
    ref, _ = _learner(None, seed=3)
    for b in bs:
        ref.update(b)
    want = {f"{net}.{n}": p.detach().clone() for net in ("actor", "critic", "target_actor")
            for n, p in getattr(ref, net).named_parameters()}
    with tempfile.TemporaryDirectory() as d:
        # (1) ZeRO W=2 -> checkpoint -> ZeRO W=2 resume
        mp.start_processes(_zero_resume_worker, args=(_free_port(), d, ""), nprocs=WORLD, join=True,
                           start_method="spawn")
        got = torch.load(os.path.join(d, "zr0.pt"), weights_only=True)
        for k in want:
            torch.testing.assert_close(got[k], want[k], rtol=1e-5, atol=1e-6)
        # (2) the ZeRO checkpoint resumed by one process without ZeRO
        one, _ = _learner(None, seed=55)
        one.load_state_dict(torch.load(os.path.join(d, "zero_sd.pt"), weights_only=True))
        one.update(bs[2])
        for net in ("actor", "critic", "target_actor"):
            for n, p in getattr(one, net).named_parameters():
                torch.testing.assert_close(p.detach(), want[f"{net}.{n}"], rtol=1e-5, atol=1e-6)
        # (3) a single-process checkpoint resumed under ZeRO W=2
        two, _ = _learner(None, seed=3)
        for b in bs[:2]:
            two.update(b)
        src = os.path.join(d, "single_sd.pt")
        torch.save(two.state_dict(), src)
        mp.start_processes(_zero_resume_worker, args=(_free_port(), d, src), nprocs=WORLD, join=True,
                           start_method="spawn")
        got = torch.load(os.path.join(d, "zr1.pt"), weights_only=True)
        for k in want:
            torch.testing.assert_close(got[k], want[k], rtol=1e-5, atol=1e-6)


def test_learner_loads_legacy_flat_checkpoint():
    """Pre-packed checkpoints (flat views of the unsharded layout) still load."""
    a, _ = _learner(None, seed=3)
    a.update(_batches(1)[0])
    sd = a.state_dict()
    legacy = {k: v for k, v in sd.items() if k != "layout"}
    for key, attr in a._NETS:
        legacy[key] = getattr(a, attr).view().clone()
    for key, opt in (("actor_opt", a.actor_opt), ("critic_opt", a.critic_opt)):
        legacy[key] = dict(sd[key], m=opt.m[:opt.fp.numel].clone(), v=opt.v[:opt.fp.numel].clone())
    b, _ = _learner(None, seed=9)
    b.load_state_dict(legacy)
    assert torch.equal(b.actor_flat.flat, a.actor_flat.flat)
    assert torch.equal(b.critic_opt.v, a.critic_opt.v)
    # a bucket-aligned (ZeRO) flat buffer is longer and shifted: refused instead of loading wrong weights
    bad = dict(legacy)
    bad["actor_opt"] = dict(legacy["actor_opt"], m=torch.cat([legacy["actor_opt"]["m"], torch.zeros(64)]))
    with pytest.raises(ValueError, match="sharded-layout"):
        b.load_state_dict(bad)


def test_dp_batched_trainer_replicas_identical():
    """Ranks step different envs (different seeds) yet hold identical parameters after every update;
    metrics are all-reduced (both ranks report the same whole-job counts)."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_trainer_worker, args=(_free_port(), d), nprocs=WORLD, join=True, start_method="spawn")
        r = [torch.load(os.path.join(d, f"t{i}.pt"), weights_only=True) for i in range(WORLD)]
    assert int(r[0]["updates"]) == 4
    assert torch.equal(r[0]["actor"], r[1]["actor"])
    assert torch.equal(r[0]["critic"], r[1]["critic"])
    assert float(r[0]["succ"]) == float(r[1]["succ"]) > 0


def _resume_worker(rank, port, out_dir, stale=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from gsc_amd.agents import SimpleDDPG
    from gsc_amd.parallel.dist import init_distributed, shutdown
    from gsc_amd.utils.experiment import setup
    info = init_distributed("cpu")
    os.chdir(ROOT)
    cfg = _cfg()
    cfg.update(episode_steps=4, nb_steps_warmup_critic=3, mem_limit=64)
    agent = os.path.join(out_dir, "agent.yaml")
    sched = os.path.join(out_dir, "sched.yaml")
    if rank == 0:
        open(agent, "w").write(yaml.safe_dump(cfg))
        open(sched, "w").write(yaml.safe_dump({"training_network_files": [ABILENE], "inference_network": ABILENE, "period": 10}))
    torch.distributed.barrier()
    svc, simc = cfg_path("service_functions", "abc.yaml"), cfg_path("config", "simulator", "sample_config.yaml")

    def make():
        h = setup(agent, ABILENE, svc, simc, sched, 7, 2, results_root=os.path.join(out_dir, f"r{rank}"))
        return SimpleDDPG(h, backend="batched", num_envs=2, device="cpu", dist_info=info, results_writers=False,
                          trainer_overrides={"batch_size": 8})

    a = make()
    a.train(1)
    path = os.path.join(out_dir, "ck.pt")
    a.save_checkpoint(path)
    torch.distributed.barrier()
    if stale:
        # a save interrupted between the ranks' writes: rank 1's file is from the previous save
        import shutil
        if rank == 1:
            shutil.copy(os.path.join(out_dir, "ck.rank1.pt"), os.path.join(out_dir, "old.pt"))
        if stale != "same_step":
            a.train(1)
        a.save_checkpoint(path)  # same_step: a re-save at the same step (equal step / episode / world size)
        if rank == 1:
            shutil.copy(os.path.join(out_dir, "old.pt"), os.path.join(out_dir, "ck.rank1.pt"))
        torch.distributed.barrier()
        b = make()
        b.load_checkpoint(path)
        torch.save({"replay_len": len(b.trainer.replay), "step": b.global_step,
                    "learning_starts": b.trainer.learning_starts}, os.path.join(out_dir, f"res{rank}.pt"))
        shutdown()
        return
    a.train(1)
    b = make()
    b.load_checkpoint(path)
    b.train(1)
    torch.save({"a_states": a.sim.states.clone(), "b_states": b.sim.states.clone(),
                "a_actor": a.learner.actor_flat.flat.clone(), "b_actor": b.learner.actor_flat.flat.clone(),
                "a_rng": a.trainer.replay.rng_state(), "b_rng": b.trainer.replay.rng_state()},
               os.path.join(out_dir, f"res{rank}.pt"))
    shutdown()


def test_dp_resume_keeps_rank_local_state():
    """Data-parallel checkpoint: rank r > 0 writes its own simulator states / replay / sampler RNG
    (checkpoint.rank{r}.pt); after resume each rank continues its own shard exactly (== the run that
    never stopped) and the shards stay distinct across ranks."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_resume_worker, args=(_free_port(), d), nprocs=WORLD, join=True, start_method="spawn")
        assert os.path.exists(os.path.join(d, "ck.rank1.pt"))
        r = [torch.load(os.path.join(d, f"res{i}.pt"), weights_only=True) for i in range(WORLD)]
    for x in r:
        assert torch.equal(x["a_states"], x["b_states"])
        assert torch.equal(x["a_actor"], x["b_actor"])
        assert torch.equal(x["a_rng"], x["b_rng"])
    assert not torch.equal(r[0]["b_states"], r[1]["b_states"])
    assert not torch.equal(r[0]["b_rng"], r[1]["b_rng"])
    assert torch.equal(r[0]["b_actor"], r[1]["b_actor"])


def test_dp_resume_rejects_stale_rank_file():
    """A rank file from another save (stamp mismatch) is not merged with rank 0's learner: that rank
    re-seeds and refills its replay ring from empty (no copy of rank 0's transitions)."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_resume_worker, args=(_free_port(), d, True), nprocs=WORLD, join=True, start_method="spawn")
        r = [torch.load(os.path.join(d, f"res{i}.pt"), weights_only=True) for i in range(WORLD)]
    assert r[0]["step"] == r[1]["step"]
    assert r[0]["replay_len"] > 0
    assert r[1]["replay_len"] == 0
    assert r[1]["learning_starts"] > r[1]["step"]


def test_dp_resume_rejects_stale_rank_file_from_same_step():
    """Two saves at the same step (e.g. a resumed run re-saving into the same directory) carry different
    nonces: a stale rank file of the first is still rejected."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_resume_worker, args=(_free_port(), d, "same_step"), nprocs=WORLD, join=True,
                           start_method="spawn")
        r = [torch.load(os.path.join(d, f"res{i}.pt"), weights_only=True) for i in range(WORLD)]
    assert r[0]["replay_len"] > 0
    assert r[1]["replay_len"] == 0


def test_dp_main_cli_train_save_exit(tmp_path):
    """main.py under torchrun (2 gloo ranks): train, the collective final checkpoint save (every rank writes
    its file, one barrier), the test episode on rank 0 and the shutdown barrier all complete; the rank files
    of the final save carry the same stamp."""
    import subprocess
    import sys
    cfg = _cfg()
    cfg.update(episode_steps=4, nb_steps_warmup_critic=3, mem_limit=64)
    agent = tmp_path / "agent.yaml"
    agent.write_text(yaml.safe_dump(cfg))
    sched = tmp_path / "sched.yaml"
    sched.write_text(yaml.safe_dump({"training_network_files": [ABILENE], "inference_network": ABILENE,
                                     "period": 10}))
    root = tmp_path / "results"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(WORLD),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "main.py"),
           str(agent), ABILENE, cfg_path("service_functions", "abc.yaml"),
           cfg_path("config", "simulator", "sample_config.yaml"), str(sched), "2", "--seed", "21", "--backend",
           "batched", "--envs", "2", "--device", "cpu", "--results-root", str(root)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    runs = [os.path.join(dp, f) for dp, _, fs in os.walk(root) for f in fs if f.startswith("checkpoint")]
    names = sorted(os.path.basename(x) for x in runs)
    assert names == ["checkpoint.pt", "checkpoint.rank1.pt"], names
    from gsc_amd.utils import checkpoint as ck
    stamps = [ck.load_checkpoint(x)["meta"]["stamp"] for x in sorted(runs)]
    assert stamps[0] == stamps[1] and stamps[0]["episode"] == 2 and stamps[0]["nonce"]
    assert "test on" in r.stdout


def test_checkpoint_format_1_rejected(tmp_path):
    from gsc_amd.utils import checkpoint as ck
    p = str(tmp_path / "old.pt")
    torch.save({"format": "gsc_amd.checkpoint/1", "meta": {}, "state": {}}, p)
    with pytest.raises(ValueError, match="no longer readable"):
        ck.load_checkpoint(p)


def _forced_worker(rank, out_dir, zero):
    """One process, GSC_DIST_FORCE=1: a world-size-1 process group; every collective is issued."""
    os.environ["GSC_DIST_FORCE"] = "1"
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    torch.set_num_threads(1)
    import torch.distributed as dist
    from gsc_amd.parallel.dist import init_distributed, shutdown
    info = init_distributed("cpu")
    assert info.forced and info.enabled and info.world_size == 1 and dist.is_initialized()
    learner, _ = _learner(info, seed=3, zero=zero)
    assert learner.zero == zero
    for b in _batches(3):
        learner.update(b)
    torch.save({f"{net}.{n}": p.detach().clone() for net in ("actor", "critic", "target_actor", "target_critic")
                for n, p in getattr(learner, net).named_parameters()}, os.path.join(out_dir, f"f{int(zero)}.pt"))
    shutdown()


@pytest.mark.parametrize("zero", [False, True])
def test_forced_world1_process_group_bit_identical(zero):
    """GSC_DIST_FORCE=1 routes the update through the data-parallel code path (collectives between the
    update stages; ZeRO-1 reduce-scatter / all-gather) over a world-size-1 group: bit-identical to the
    process-local learner (the GPU twin runs the same over RCCL: tests/test_gpu_dp.py)."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_forced_worker, args=(d, zero), nprocs=1, join=True, start_method="spawn")
        got = torch.load(os.path.join(d, f"f{int(zero)}.pt"), weights_only=True)
    nt = torch.get_num_threads()
    torch.set_num_threads(1)   # the worker's CPU GEMM reduction order
    try:
        ref, _ = _learner(None, seed=3)
        for b in _batches(3):
            ref.update(b)
    finally:
        torch.set_num_threads(nt)
    for net in ("actor", "critic", "target_actor", "target_critic"):
        for n, p in getattr(ref, net).named_parameters():
            assert torch.equal(got[f"{net}.{n}"], p.detach()), f"{net}.{n}"


def _bf16_worker(rank, port, out_dir, big):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from gsc_amd.parallel.dist import GradReduce, init_distributed, shutdown
    info = init_distributed("cpu")
    if big:
        # a config-5-sized gradient (the syn200 actor: ~185 M fp32 values), bf16 vs fp32 sums
        g = torch.Generator().manual_seed(100 + rank)
        n = big
        grad = torch.randn(n, generator=g) * 1e-3
        ref = grad.clone()
        GradReduce(ref, None).wait()
        got = grad.clone()
        GradReduce(got, torch.zeros(n, dtype=torch.bfloat16)).wait()
        rel = ((got - ref).abs().max() / ref.abs().max()).item()
        torch.save({"rel": torch.tensor(rel)}, os.path.join(out_dir, f"big{rank}.pt"))
    else:
        from gsc_amd.agents import Batch
        os.environ["GSC_DP_GRAD_BF16"] = "1"
        learner, _ = _learner(info, seed=3)
        assert learner.grad_bf16
        for b in _batches(3):
            sl = slice(rank * B_PER_RANK, (rank + 1) * B_PER_RANK)
            learner.update(Batch(*(t[sl] for t in b)))
        torch.save({"actor": learner.actor_flat.flat.clone(), "critic": learner.critic_flat.flat.clone()},
                   os.path.join(out_dir, f"bf{rank}.pt"))
    shutdown()


def test_dp_bf16_gradient_allreduce_close_to_fp32():
    """GSC_DP_GRAD_BF16=1: replicas stay bit-identical, and 3 updates stay within bf16
    rounding of the fp32-reduced single-process update (Adam's step is ~lr per element, so a relative
    gradient error of ~2^-8 moves a parameter by far less than lr)."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_bf16_worker, args=(_free_port(), d, 0), nprocs=WORLD, join=True, start_method="spawn")
        r = [torch.load(os.path.join(d, f"bf{i}.pt"), weights_only=True) for i in range(WORLD)]
    assert torch.equal(r[0]["actor"], r[1]["actor"]) and torch.equal(r[0]["critic"], r[1]["critic"])
    ref, _ = _learner(None, seed=3)
    for b in _batches(3):
        ref.update(b)
    for k, fp in (("actor", ref.actor_flat), ("critic", ref.critic_flat)):
        d = (r[0][k] - fp.flat).abs().max().item()
        assert d < 3 * 1e-3, (k, d)   # 3 updates of at most ~lr each; fp32 reduction differs by ~1e-7


@pytest.mark.slow
def test_dp_bf16_gradient_allreduce_config5_size():
    """The bf16 all-reduce of a config-5-sized gradient (185 M values, 2 gloo ranks): max error relative
    to the largest sum within bf16 rounding of the inputs and of the sum (2^-8 each)."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_bf16_worker, args=(_free_port(), d, 185_000_000), nprocs=WORLD, join=True,
                           start_method="spawn")
        rel = [float(torch.load(os.path.join(d, f"big{i}.pt"), weights_only=True)["rel"]) for i in range(WORLD)]
    assert max(rel) < 2 ** -7, rel
