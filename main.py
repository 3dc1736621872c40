#!/usr/bin/env python
"""Training + test CLI (reference ``main.py:16-76``, same positionals and options).

    python main.py <agent_config> <network> <service> <sim_config> <scheduler> <episodes> [options]

Reference options: ``--seed`` (random default), ``-t/--test <run id>`` (test a trained run
only), ``-w/--weights <file|dir>`` (resume; the reference parses it but never loads it),
``-a/--append-test`` (test into ``<run>/test-<time>_seed<seed>/``), ``-v``, ``-b/--best`` (test
the best earlier run), ``-ss/--sim-seed``, ``-gs/--gen-scenario <sim_config>`` (an extra test
on a different simulator config).

New options: ``--backend auto|oracle|batched`` (auto = batched device simulator on a GPU, the
scalar reference-equivalent loop on CPU), ``--envs`` (batched envs per GPU), ``--device``,
``--checkpoint-every <episodes>``, ``--results-root``, ``--no-test``.  Multi-GPU:
``python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 main.py ...``
(one process per GPU, RCCL all-reduce; rank 0 writes the result directory).

Outputs (``results/<agent>/<scheduler>/<service>/<simcfg>/<time>_seed<seed>/``):
``trained_actor.pt`` (state_dict + config header), ``agent_helper.obj`` (JSON), ``checkpoint.pt``,
``rewards.csv``, ``metrics.jsonl``, ``result.yaml``, ``training.log``, input copies, test CSVs.
"""
from __future__ import annotations

import os
import random
import sys

import click

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _resolve_weights(path: str):
    """-> (kind, file) with kind in {"checkpoint", "actor"}."""
    if os.path.isdir(path):
        for kind, name in (("checkpoint", "checkpoint.pt"), ("actor", "trained_actor.pt")):
            f = os.path.join(path, name)
            if os.path.exists(f):
                return kind, f
        raise click.BadParameter(f"{path} contains neither checkpoint.pt nor trained_actor.pt")
    import torch
    d = torch.load(path, map_location="cpu", weights_only=True)
    fmt = d.get("format", "") if isinstance(d, dict) else ""
    if fmt.startswith("gsc_amd.checkpoint"):
        return "checkpoint", path
    if fmt.startswith("gsc_amd.actor"):
        return "actor", path
    raise click.BadParameter(f"{path}: unknown weights format")


def select_best_agent(result_dir: str, last_n: int = 10):
    """Run id in ``result_dir`` with the best mean return over its last ``last_n`` episodes (``rewards.csv``).

    Reference ``select_best_agent`` (src/rlsp/agents/main.py:89-113) reads an ``episode_reward.csv``
    nobody writes; this reads the ``rewards.csv`` every run here writes."""
    best, best_id = None, None
    if not os.path.isdir(result_dir):
        return None
    for run in sorted(os.listdir(result_dir)):
        f = os.path.join(result_dir, run, "rewards.csv")
        if run == "best" or not os.path.exists(os.path.join(result_dir, run, "trained_actor.pt")) or not os.path.exists(f):
            continue
        with open(f) as fh:
            vals = [float(x) for x in fh.read().split() if x.strip()]
        if not vals:
            continue
        score = sum(vals[-last_n:]) / len(vals[-last_n:])
        if best is None or score > best:
            best, best_id = score, run
    click.echo(f"Best agent found: {best_id} with avg reward of {best}")
    return best_id


@click.command(context_settings=dict(help_option_names=["-h", "--help"]))
@click.argument("agent_config", type=click.Path(exists=True))
@click.argument("network", type=click.Path(exists=True))
@click.argument("service", type=click.Path(exists=True))
@click.argument("sim_config", type=click.Path(exists=True))
@click.argument("scheduler", type=click.Path(exists=True))
@click.argument("episodes", type=int)
@click.option("--seed", type=int, default=None, help="Random seed for the environment and the agent (default: random 1000-9999).")
@click.option("-t", "--test", default=None, help="Run id whose trained actor is tested (no training).")
@click.option("-w", "--weights", default=None, help="Resume from a checkpoint.pt / trained_actor.pt (file or run dir).")
@click.option("-a", "--append-test", is_flag=True, help="Append a test run of the trained agent in its own subdir.")
@click.option("-v", "--verbose", is_flag=True, help="Console logger at DEBUG.")
@click.option("-b", "--best", is_flag=True, help="Test the best of the runs trained so far.")
@click.option("-ss", "--sim-seed", type=int, default=None, help="Simulator seed.")
@click.option("-gs", "--gen-scenario", type=click.Path(exists=True), default=None,
              help="Different simulator config for an additional scenario test.")
@click.option("--backend", type=click.Choice(["auto", "oracle", "batched"]), default="auto")
@click.option("--envs", type=int, default=256, help="Batched environments per GPU.")
@click.option("--device", default=None, help="cuda | cpu (default: cuda when available).")
@click.option("--checkpoint-every", type=int, default=0, help="Write checkpoint.pt every N episodes (0: at the end).")
@click.option("--results-root", default="results")
@click.option("--no-test", is_flag=True, help="Skip the greedy test episode after training.")
@click.option("--checkpoint-replay", type=click.Choice(["auto", "yes", "no"]), default="auto",
              help="Include the replay ring in checkpoint.pt (auto: if <= 1 GiB).")
def cli(agent_config, network, service, sim_config, scheduler, episodes, seed, test, weights, append_test, verbose,
        best, sim_seed, gen_scenario, backend, envs, device, checkpoint_every, results_root, no_test,
        checkpoint_replay):
    """GSC training and testing (GATv2 + DDPG on coord-sim), MI355X-native."""
    import torch

    from gsc_amd.agents import SimpleDDPG
    from gsc_amd.parallel.dist import init_distributed, shutdown, sync_string
    from gsc_amd.utils import experiment as xp
    from gsc_amd.utils.checkpoint import save_agent_helper

    if seed is None:
        seed = random.randint(1000, 9999)
    dev_type = device or ("cuda" if torch.cuda.is_available() else "cpu")
    info = init_distributed(dev_type)
    if dev_type == "cuda":
        torch.cuda.set_device(info.local_rank)
    stamp = sync_string(xp.DATETIME)           # one result directory for all ranks
    seed = int(sync_string(str(seed)))
    if best:
        base = os.path.join(results_root, xp.get_base_path(agent_config, scheduler, service, sim_config))
        test = select_best_agent(base)
        if test is None:
            raise click.ClickException(f"no trained runs under {base}")
    h = xp.setup(agent_config, network, service, sim_config, scheduler, seed, episodes, weights, verbose, test=test,
                 append_test=append_test, sim_seed=sim_seed, gen_scenario=gen_scenario, results_root=results_root,
                 datetime_str=stamp, write_files=info.is_main)
    agent = SimpleDDPG(h, backend=backend, num_envs=envs, device=dev_type if dev_type == "cpu" else None,
                       dist_info=info, checkpoint_every=checkpoint_every)
    agent.checkpoint_replay = checkpoint_replay
    log = xp.logger
    if test and not append_test:
        actor_file = os.path.join(h.weights_path, "trained_actor.pt")
        log.info(f"testing {actor_file}")
        agent.load_actor_weights(actor_file)
    else:
        if weights:
            kind, f = _resolve_weights(weights)
            log.info(f"resuming from {kind} {f}")
            agent.load_checkpoint(f) if kind == "checkpoint" else agent.load_actor_weights(f)
        h.result.runtime_start()
        stats = agent.train(episodes)
        h.result.runtime_stop()
        log.info(f"training done: {stats}")
        # the checkpoint save is collective (data parallel: every rank writes its rank-local trainer state
        # and the ranks meet at a barrier); the actor / helper / result files are rank 0's
        agent.save_actor(os.path.join(h.config_dir, "trained_actor.pt"))
        agent.save_checkpoint(os.path.join(h.config_dir, "checkpoint.pt"))
        if info.is_main:
            save_agent_helper(os.path.join(h.config_dir, "agent_helper.obj"), h)
            h.result.agent_config = dict(h.config)
            h.result.write_to_file(h.result_file)
    if info.is_main and not no_test:
        if append_test:
            h.config_dir = os.path.join(h.config_dir, f"test-{stamp}_seed{seed}") + os.sep
            os.makedirs(h.config_dir, exist_ok=True)
        res = agent.test()
        xp.write_yaml(os.path.join(h.config_dir, "test_result.yaml"), res)
        click.echo(f"test on {os.path.basename(h.schedule['inference_network'])}: return {res['return']:.3f} "
                   f"success ratio {res['success_ratio']:.3f}")
        if gen_scenario:
            h.sim_config_path = gen_scenario
            h.config_dir = os.path.join(h.config_dir, "gen-scenario") + os.sep
            os.makedirs(h.config_dir, exist_ok=True)
            res = agent.test()
            xp.write_yaml(os.path.join(h.config_dir, "test_result.yaml"), res)
            click.echo(f"generalisation scenario {os.path.basename(gen_scenario)}: success {res['success_ratio']:.3f}")
    agent.close()
    shutdown()


if __name__ == "__main__":
    cli()
