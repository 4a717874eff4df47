"""C5 benchmark: 2-hop expand + re-score inside the RL environment loop (SURVEY §8, configs[4]).

Builds a HotpotQA-distractor-shaped graph (87,000 entities + 3,000 summaries indexed,
2 belongs_to parents per entity, ~2 related_to per summary, 40,000 hyperedges x ~3.8
participants, unindexed) with the seeded corpus vectors of ah_rag.synthetic written straight into
the vector store (no encoder weights offline), then times
  * vec:    VecAHRAGGymEnv with E environments: one batched reset (dense top-5 + expansion +
            rerank for all E queries) and `steps` batched steps of random valid actions;
  * single: the drop-in AHRAGGymEnv stepped one environment at a time (B = 1 per call), the
            reference's own loop shape (policy_ppo.py:145,163-214) on the device graph: one
            untimed pass over its episodes, then the median of three timed passes (each reported:
            a pass is ~20 ms, so one host stall moves a single pass by tens of percent).
Replicas per GPU: --gpus N runs one process per GPU (spawned by this script, or
under torch.distributed.run), the graph and corpus replicated, the --envs environments
partitioned over the ranks; no collective on the data path (the job time is the slowest rank's).
Prints one JSON line. Usage: python tools/bench_env.py [--gpus 8] [--envs 1024] [--steps 6] [--episodes 5]
[--cpu-seconds 10]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ah_rag.agent.gym_env import AHRAGGymEnv  # noqa: E402
from ah_rag.agent.vec_env import VecAHRAGGymEnv  # noqa: E402
from ah_rag.distributed import launch  # noqa: E402
from ah_rag.synthetic import HOTPOT_90K, SyntheticCorpus, build_hotpot_graph, install_vectors  # noqa: E402


def random_actions(rng, masks):
    return [int(rng.choice(np.flatnonzero(np.asarray(m)))) for m in masks]


def random_actions_batch(rng, masks: np.ndarray) -> np.ndarray:
    """A uniformly random valid action per row of an [E, 6] mask (the batched policy's draw)."""
    u = rng.random(masks.shape) * (masks > 0)
    return np.argmax(u, axis=1)


def single_reset(env: AHRAGGymEnv, hg, query: str, qvec: np.ndarray):
    """AHRAGGymEnv.reset(query) with a precomputed query vector (no encoder weights offline): the
    same GraphEnvironment.reset + semantic_anchor steps (environment.py:155-241), the search at B = 1."""
    ge = env.env
    env._query, env._cur_step = query, 0
    ge.last_query, ge.last_results, ge.step_count = None, None, 0
    ge.selection_set.clear()
    ge.frontier_set.clear()
    ge.step_count += 1
    ge.last_query = query
    cluster = hg.search_batch([query], top_k=5, member_top_m=5, return_cluster=True, query_vectors=qvec)[0]
    obs, _ = ge._anchor_result(query, 5, cluster, 0.0)
    return env._finish_reset(obs)


def reference_loop(hg, tmp: str, steps: int, n_envs: int = 4, budget_s: float = 3.0, seed: int = 20251003) -> dict:
    """The reference's PPO environment loop unchanged in shape (scripts/train_ppo.py:25-26,
    policy_ppo.py:145,163-205): `n_envs` environments built by AHRAGGymEnv(graph_dir=...) from a
    saved graph directory, then rounds of {reset every env with its question (the encoder in the
    loop: AHR_ENCODER=hash, no weights offline), step each env one after another with a random
    valid action until done}. Construction times are reported per environment (the first loads the
    graph; the rest share it and its device structures, HierarchicalGraph.load_shared); the first
    round (device graph, index upload, kernels' first calls) is reported and not timed."""
    gdir = os.path.join(tmp, "graph_ref")
    vi = hg.G.graph["vector_index"]
    model = vi.get("model")
    vi["model"] = "all-mpnet-base-v2"  # a 768-wide name: the hash encoder then matches the corpus width
    t0 = time.perf_counter()
    try:
        hg.save(gdir)
    finally:
        vi["model"] = model
    save_s = time.perf_counter() - t0
    prev = os.environ.get("AHR_ENCODER")
    os.environ["AHR_ENCODER"] = "hash"
    rng = np.random.default_rng(seed)
    try:
        ctor_s, envs = [], []
        for _ in range(n_envs):
            t = time.perf_counter()
            envs.append(AHRAGGymEnv(graph_dir=gdir, max_steps=steps))
            ctor_s.append(time.perf_counter() - t)

        def one_round(r: int) -> int:
            n = 0
            for e, env in enumerate(envs):
                env.reset(f"question {r}.{e} about the corpus")
            n += len(envs)
            for env in envs:
                done, k = False, 0
                while not done and k < steps:
                    a = random_actions(rng, [env.get_action_mask()])[0]
                    _, _, done, _ = env.step(a)
                    n += 1
                    k += 1
            return n
        t = time.perf_counter()
        one_round(0)
        torch.cuda.synchronize()
        first_s = time.perf_counter() - t
        n_steps, r, t = 0, 1, time.perf_counter()
        while True:
            n_steps += one_round(r)
            r += 1
            if time.perf_counter() - t >= budget_s:
                break
        dt = time.perf_counter() - t
    finally:
        if prev is None:
            os.environ.pop("AHR_ENCODER", None)
        else:
            os.environ["AHR_ENCODER"] = prev
    shared = all(env.env.hg is envs[0].env.hg for env in envs)
    return {"env_steps_per_s": round(n_steps / dt, 1), "rounds": r - 1, "env_steps": n_steps,
            "n_envs": n_envs, "ctor_s": [round(x, 4) for x in ctor_s], "first_round_s": round(first_s, 3),
            "graph_save_s": round(save_s, 2), "graph_shared": shared,
            "what": (f"AHRAGGymEnv(graph_dir=...) x {n_envs} from a saved graph directory, then rounds of reset-all + "
                     "each env stepped to done one after another (policy_ppo.py:145,163-205), random valid actions, "
                     "hash encoder for the reset queries, fp32 index; env steps = resets + steps")}


def measure(dev, envs: int, steps: int, single: int = 64, rank: int = 0, world: int = 1, total_envs=None,
            backend: str = "nccl", episodes: int = 5, cpu_baseline_fn=None) -> dict:
    """One rank's C5 measurement: build the graph, then a warm-up episode and `episodes` timed
    batched VecAHRAGGymEnv episodes of `envs` environments (reset + `steps` steps of random valid
    actions), with the device time of every search / expansion pass (HIP events, ah_rag.devtime)
    beside the wall time; on rank 0, `single` environments stepped one by one and, with
    cpu_seconds > 0, the host restatement of the reference loop (cpu_env_baseline). The job time is
    the slowest rank's when world > 1 (an all-reduce of the timed episodes, the only collective)."""
    from ah_rag import devtime
    total_envs = envs if total_envs is None else total_envs
    rng = np.random.default_rng(20251003 + rank)
    t0 = time.perf_counter()
    corpus = SyntheticCorpus(HOTPOT_90K, dev)
    vectors = corpus.rows().cpu().numpy()
    hg, ids = build_hotpot_graph(corpus, np.random.default_rng(20251003))  # the same graph on every rank
    tmp = tempfile.mkdtemp(prefix="ahr_env_")
    install_vectors(hg, ids, vectors, os.path.join(tmp, "vector_db"))
    q, _ = corpus.queries(envs, corpus.rows(), salt=rank)
    qv = q.cpu().numpy()
    # the batched resets take the query vectors where a GPU encoder leaves them, resident in HBM
    # (the bench contract's inputs: no 3 MB host-to-device staging per reset); the one-environment
    # loops below take host vectors, as the drop-in search() does
    q_dev = q.contiguous()
    queries = [f"query {rank}.{i}" for i in range(envs)]
    t_build = time.perf_counter() - t0

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    venv = VecAHRAGGymEnv(n_envs=envs, max_steps=steps + 1, graph=hg)
    # warm-up episode: device graph, index, expansion kernels, host caches
    venv.reset(queries, query_vectors=q_dev)
    for _ in range(steps):
        venv.step(random_actions_batch(rng, venv.action_masks()))
    barrier()
    ep_times, reset_wall, step_wall = [], [], [[] for _ in range(steps)]
    spans = {"reset": [], "step": []}  # (first, last) span index per phase
    with devtime.recording() as pairs:
        t1 = time.perf_counter()
        for _ in range(episodes):
            te = time.perf_counter()
            n0 = len(pairs)
            venv.reset(queries, query_vectors=q_dev)
            reset_wall.append(time.perf_counter() - te)
            spans["reset"].append((n0, len(pairs)))
            for j in range(steps):
                acts = random_actions_batch(rng, venv.action_masks())  # the policy's batched draw
                ts = time.perf_counter()
                n0 = len(pairs)
                venv.step(acts)
                step_wall[j].append(time.perf_counter() - ts)
                spans["step"].append((n0, len(pairs)))
            ep_times.append(time.perf_counter() - te)
        barrier()
        vec_time = time.perf_counter() - t1
        dev_ms = {ph: [devtime.total_ms(pairs[a:b]) for a, b in v] for ph, v in spans.items()}
    if world > 1:  # job time = the slowest rank
        t = torch.tensor([vec_time], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        vec_time = float(t.item())
    vec_steps = episodes * total_envs * (1 + steps)  # all ranks' environments
    # (the masks and action draws between steps are the caller's policy, outside the step walls)
    reset_ms, step_ms = np.mean(reset_wall) * 1e3, float(np.sum([np.mean(w) for w in step_wall])) * 1e3 / steps
    dev_reset, dev_step = float(np.mean(dev_ms["reset"])), float(np.mean(dev_ms["step"]))

    single_rate = search_s = None
    if rank == 0 and single > 0:
        # single-environment loop (B = 1 per search / expansion), a subset of the same queries
        n1 = min(single, envs)
        env = AHRAGGymEnv(max_steps=steps + 1, graph=hg)
        env.env.logging_enabled = False
        for i in range(2):  # warm-up episodes: every action kind's first call, the host allocator
            single_reset(env, hg, queries[-1 - i], qv[-1 - i:len(qv) - i])
            for a in (0, 1, 2, 3, 4, 0):
                env.step(a if env.get_action_mask()[a] else random_actions(rng, [env.get_action_mask()])[0])
        torch.cuda.synchronize()

        def single_pass():
            ts = time.perf_counter()
            for i in range(n1):
                # reset with a precomputed vector (the search at B = 1)
                single_reset(env, hg, queries[i], qv[i:i + 1])
                for _ in range(steps):
                    env.step(random_actions(rng, [env.get_action_mask()])[0])
            return n1 * (1 + steps) / (time.perf_counter() - ts)
        # one untimed pass over the same episodes (first visits: the node briefs, the per-shape
        # buffers), then three timed passes; the median is the rate, all three are reported
        single_pass()
        single_passes = [round(single_pass(), 1) for _ in range(3)]
        single_rate = float(np.median(single_passes))
        # the drop-in search itself: HierarchicalGraph.search's body at B = 1 (dense top-5 + expansion
        # + rerank + the result dicts, return_cluster=False) with a precomputed query vector
        n_s = min(256, envs)
        for i in range(8):
            hg.search_batch([queries[i]], top_k=5, member_top_m=5, query_vectors=qv[i:i + 1])
        torch.cuda.synchronize()

        def search_pass():
            ts = time.perf_counter()
            for i in range(n_s):
                hg.search_batch([queries[i]], top_k=5, member_top_m=5, query_vectors=qv[i:i + 1])
            return (time.perf_counter() - ts) / n_s
        # three timed passes (the host CPU of a shared box is noisy, as the single-env passes show):
        # the median is the figure, all three are reported
        search_passes = [search_pass() for _ in range(3)]
        search_s = float(np.median(search_passes))
    ref_loop = reference_loop(hg, tmp, steps) if rank == 0 and single > 0 else None
    cpu = None
    if rank == 0 and cpu_baseline_fn is not None:
        cpu = cpu_baseline_fn(hg, ids, vectors, qv, steps)
    return {
        "metric": f"env steps/sec (reset + steps, 2-hop expand + rerank), C5 on {world} MI355X",
        "n_gpus": world, "envs": total_envs, "envs_per_gpu": envs, "steps_per_episode": steps,
        "episodes": episodes,
        "vec_env_steps_per_s": round(vec_steps / vec_time, 1),
        "episode_s": round(vec_time / episodes, 4),
        "episodes_s": [round(t, 4) for t in ep_times],
        "vec_step_only_per_s_rank0": round(envs / (step_ms * 1e-3), 1),
        "vec_reset_ms_rank0": round(reset_ms, 2),
        "vec_step_ms_rank0": [round(float(np.mean(w)) * 1e3, 2) for w in step_wall],
        "device_host_split_rank0": {
            "reset_wall_ms": round(reset_ms, 3), "reset_device_ms": round(dev_reset, 3),
            "reset_host_ms": round(reset_ms - dev_reset, 3),
            "step_wall_ms": round(step_ms, 3), "step_device_ms": round(dev_step, 3),
            "step_host_ms": round(step_ms - dev_step, 3),
            "how": "device = HIP-event spans around every search / expansion pass (ah_rag.devtime) on the "
                   "launch stream, summed; host = wall - device; means over the timed episodes"},
        "single_env_steps_per_s": single_rate,
        "single_env_passes": single_passes if rank == 0 and single > 0 else None,
        "dropin_search_b1": None if search_s is None else {
            "calls_per_s": round(1.0 / search_s, 1), "ms_per_call": round(search_s * 1e3, 4),
            "ms_per_call_passes": [round(t * 1e3, 4) for t in search_passes],
            "what": "HierarchicalGraph.search_batch([q], top_k=5, return_cluster=False) wall time per "
                    "call at B = 1 with a precomputed query vector (the body of the drop-in search(); "
                    "fp32 index, 90k rows), 256 calls after 8 warm-up calls; the median of three passes"},
        "reference_loop": ref_loop,
        "cpu_baseline": cpu,
        "graph": {"nodes": hg.G.number_of_nodes(), "edges": hg.G.number_of_edges(), "indexed": len(ids)},
        "build_s": round(t_build, 1), "parallelism": f"replicas{world} (environments partitioned, no collective)",
        "data": "synthetic HotpotQA-distractor-shaped graph (SURVEY §8d), seeded corpus vectors, random valid actions; "
                "batched resets take their query vectors resident in HBM (a GPU encoder's output), the "
                "one-environment loops host vectors",
    }


def run(a) -> None:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        # replicas: no collective on the data path, only the timing reduction
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    envs = a.envs // world + (1 if rank < a.envs % world else 0)  # environments partitioned over ranks
    cpu_fn = None
    if a.cpu_seconds > 0:
        from bench import cpu_env_baseline
        cpu_fn = lambda *x: cpu_env_baseline(*x, budget_s=a.cpu_seconds)  # noqa: E731
    out = measure(dev, envs, a.steps, a.single, rank, world, a.envs, a.backend, a.episodes, cpu_fn)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--envs", type=int, default=1024, help="environments of the whole job")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--single", type=int, default=64, help="environments stepped one by one (rank 0)")
    ap.add_argument("--episodes", type=int, default=5, help="timed episodes after the warm-up one")
    ap.add_argument("--cpu-seconds", type=float, default=0.0, help="host baseline budget (rank 0; 0 = off): bench.cpu_env_baseline")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl")
    a = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        launch(a.gpus, run, (a,))  # one process per GPU, spawned before any GPU call
        return
    run(a)


if __name__ == "__main__":
    main()
