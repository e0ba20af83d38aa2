"""Worker for tests/test_gpu_dist.py: DeviceGA generations with the
population sharded over WORLD_SIZE ranks (gloo; every rank on cuda:0), rank 0
saves the final state.

usage: python _dist_ga_worker.py OUT_DIR            (small: [6,8,3], P 101, 3 generations)
       python _dist_ga_worker.py OUT_DIR config4    (BASELINE config 4: [6,64,3], P 524 288,
                                                     self-play vs P/4 hall of fame, 2 generations)
       python _dist_ga_worker.py OUT_DIR wide       (BASELINE config 5's [6,512,512,3], f32, P 256,
                                                     self-play vs a 64-row hall, 2 generations;
                                                     wide_balanced: the length-balanced shards)
       python _dist_ga_worker.py OUT_DIR slices     ([6,8,3], P 96, hall of 3 < 4 row blocks)
At world > 1 DeviceGA varies only each rank's shard (shard_vary).
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "neuro-genetic-pong-self-play_amd"))


def main(out_dir, mode="small"):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo")
    from pong_amd import device as D
    from pong_amd.evolve import DeviceGA
    dev = torch.device("cuda", 0)
    if mode == "config4":
        P = 524288
        # bench.py's schedule: each 65 536-row block plays its slice of the hall
        ga = DeviceGA([6, 64, 3], P, device=dev, schedule="selfplay", seed=4, hof_block_rows=65536)
        ga.initialize("normal", 3.0)
        sample = {}

        def keep(g, rows, opponents, res):  # the last evaluation's inputs for 48 of this rank's rows
            n = res.fitness.shape[0]
            rng = np.random.default_rng(g)
            pick = np.sort(rng.choice(n, size=min(48, n), replace=False))
            pt = torch.as_tensor(pick, device=dev)
            r = ga.last_rows[pt].long() if ga.last_rows is not None else pt  # rows: full offspring / the shard
            kind, opp, mult = ga.eval_schedule(g)  # (opp indexes `opponents`: the hall or this rank's slice)
            o = opp[pt].cpu().numpy()
            used = np.unique(o)  # only the hall-of-fame rows these games play
            opp_rows = (opponents[torch.as_tensor(used, device=dev)].double().cpu().numpy()
                        if opponents is not None else None)
            sample.update(genomes=rows[r].double().cpu().numpy(), kind=kind[pt].cpu().numpy(),
                          opp=np.searchsorted(used, o).astype(np.int32), mult=mult[pt].cpu().numpy(),
                          opponents=opp_rows,
                          fitness=res.fitness[pt].cpu().numpy(), frames=res.frames[pt].cpu().numpy(),
                          played=(torch.arange(n, device=dev)[pt] < (ga.last_count[0] if ga.last_count is not None
                                                                      else n)).cpu().numpy())
        ga.on_evaluate = keep
        ga.step()              # generation 0: the initial evaluation
        ga.profile = {}        # generation 1 phases (synchronised per phase)
        t0 = time.perf_counter()
        ga.step()
        torch.cuda.synchronize()
        step_ms = (time.perf_counter() - t0) * 1e3
        phases = dict(ga.profile)
        ga.profile = None
        # sharded variation: each rank holds its shard's rows; the hashes are all-gathered
        h = ga.population_hash().cpu().numpy()
        if not dist.is_initialized() or dist.get_rank() == 0:
            os.makedirs(out_dir, exist_ok=True)
            np.save(os.path.join(out_dir, "pop_hash.npy"), h)
            np.save(os.path.join(out_dir, "fitness.npy"), ga.fitness.cpu().numpy())
            np.save(os.path.join(out_dir, "hof_hash.npy"), D.row_hash(ga.hall_of_fame, ga.G).cpu().numpy())
            np.save(os.path.join(out_dir, "hof_fitness.npy"), ga.hof_member_fitness)
            np.savez(os.path.join(out_dir, "sample.npz"), **{k: v for k, v in sample.items() if v is not None})
            with open(os.path.join(out_dir, "profile.json"), "w") as fh:
                json.dump({"world": world, "rank_rows": ga.hi - ga.lo, "generation1_ms": step_ms,
                           "generation1_phases_ms": phases, "logbook": ga.logbook}, fh)
    elif mode in ("wide", "wide_balanced"):
        # BASELINE config 5's network [6,512,512,3] (f32 genomes, k_wide) at a small
        # population, self-play vs the hall of fame: the 1 -> N strong-scaling split
        P = 256
        ga = DeviceGA([6, 512, 512, 3], P, hof_size=64, tournsize=64, dtype=torch.float32, device=dev,
                      schedule="selfplay", seed=9)
        ga.balance_shards = mode == "wide_balanced"
        ga.initialize("normal", 3.0)
        sample = {}

        def keep(g, rows, opponents, res):  # 4 of this rank's evaluated genomes, for an oracle replay
            n = res.fitness.shape[0]
            played = int(ga.last_count[0]) if ga.last_count is not None else n
            pick = np.arange(min(4, played))
            pt = torch.as_tensor(pick, device=dev)
            r = ga.last_rows[pt].long() if ga.last_rows is not None else pt
            kind, opp, mult = ga.eval_schedule(g)
            o = opp[pt].cpu().numpy()
            used = np.unique(o)
            sample.update(genomes=rows[r].double().cpu().numpy(), kind=kind[pt].cpu().numpy(),
                          opp=np.searchsorted(used, o).astype(np.int32), mult=mult[pt].cpu().numpy(),
                          opponents=(opponents[torch.as_tensor(used, device=dev)].double().cpu().numpy()
                                     if opponents is not None else np.zeros((1, ga.G))),  # (generation 0: no hall yet)
                          fitness=res.fitness[pt].cpu().numpy(), frames=res.frames[pt].cpu().numpy())
        ga.on_evaluate = keep
        ga.run(2)
        h = ga.population_hash().cpu().numpy()
        if not dist.is_initialized() or dist.get_rank() == 0:
            os.makedirs(out_dir, exist_ok=True)
            np.save(os.path.join(out_dir, "pop_hash.npy"), h)
            np.save(os.path.join(out_dir, "fitness.npy"), ga.fitness.cpu().numpy())
            np.save(os.path.join(out_dir, "hof_hash.npy"), D.row_hash(ga.hall_of_fame, ga.G).cpu().numpy())
            np.save(os.path.join(out_dir, "hof_fitness.npy"), ga.hof_member_fitness)
            np.savez(os.path.join(out_dir, "sample.npz"), **sample)
            with open(os.path.join(out_dir, "profile.json"), "w") as fh:
                json.dump({"world": world, "logbook": ga.logbook}, fh)
    elif mode == "slices":
        # a sliced hall (pg_schedule_args.hof_slices) with fewer members than row
        # blocks: P = 96 in 4 blocks of 24, a 3-member hall -> K = 3 slices, and
        # block 3 plays slice 3 mod 3 = 0 (round-5 review: rank 3 had passed an
        # empty slice); each of 4 ranks holds one block
        ga = DeviceGA([6, 8, 3], 96, hof_size=3, tournsize=9, device=dev, schedule="selfplay", seed=21,
                      hof_block_rows=24)
        ga.initialize("normal", 2.0)
        ga.run(3)
        pop = ga.population_full().cpu().numpy()
        if not dist.is_initialized() or dist.get_rank() == 0:
            os.makedirs(out_dir, exist_ok=True)
            np.save(os.path.join(out_dir, "population.npy"), pop)
            np.save(os.path.join(out_dir, "fitness.npy"), ga.fitness.cpu().numpy())
            np.save(os.path.join(out_dir, "hof.npy"), ga.hall_of_fame.cpu().numpy())
            np.save(os.path.join(out_dir, "hof_fitness.npy"), ga.hof_member_fitness)
            np.save(os.path.join(out_dir, "rows.npy"), np.array([ga.lo, ga.hi, ga.hof_slices,
                                                                 -1 if ga._slice is None else ga._slice]))
    else:
        ga = DeviceGA([6, 8, 3], 101, hof_size=20, tournsize=9, device=dev, schedule="reference", seed=77)
        ga.initialize("normal", 2.0)
        ga.run(3)
        pop = ga.population_full().cpu().numpy()  # (sharded variation: an all-gather of the shards' rows)
        if ga._sharded():  # a rank holds only its shard current: the plain view refuses
            try:
                ga.population
            except RuntimeError:
                pass
            else:
                raise AssertionError("DeviceGA.population returned rows of a sharded run")
            assert ga.shard_rows().shape[0] == ga.hi - ga.lo
        if not dist.is_initialized() or dist.get_rank() == 0:
            os.makedirs(out_dir, exist_ok=True)
            np.save(os.path.join(out_dir, "population.npy"), pop)
            np.save(os.path.join(out_dir, "fitness.npy"), ga.fitness.cpu().numpy())
            np.save(os.path.join(out_dir, "hof.npy"), ga.hall_of_fame.cpu().numpy())
            np.save(os.path.join(out_dir, "hof_fitness.npy"), ga.hof_member_fitness)
            np.save(os.path.join(out_dir, "rows.npy"), np.array([ga.lo, ga.hi]))
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "small")
