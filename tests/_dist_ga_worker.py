"""Worker for tests/test_gpu_dist.py: a few DeviceGA generations with the
population sharded over WORLD_SIZE ranks (gloo; every rank on cuda:0), rank 0
saves the final state.  usage: python _dist_ga_worker.py OUT_DIR"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "neuro-genetic-pong-self-play_amd"))


def main(out_dir):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo")
    from pong_amd.evolve import DeviceGA
    ga = DeviceGA([6, 8, 3], 101, hof_size=20, tournsize=9, device=torch.device("cuda", 0),
                  schedule="reference", seed=77)
    ga.initialize("normal", 2.0)
    ga.run(3)
    if not dist.is_initialized() or dist.get_rank() == 0:
        os.makedirs(out_dir, exist_ok=True)
        np.save(os.path.join(out_dir, "population.npy"), ga.population.cpu().numpy())
        np.save(os.path.join(out_dir, "fitness.npy"), ga.fitness.cpu().numpy())
        np.save(os.path.join(out_dir, "hof.npy"), ga.hall_of_fame.cpu().numpy())
        np.save(os.path.join(out_dir, "hof_fitness.npy"), ga.hof_member_fitness)
        np.save(os.path.join(out_dir, "rows.npy"), np.array([ga.lo, ga.hi]))
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
