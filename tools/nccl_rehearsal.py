"""Exercise bench.py's RCCL code path (init, counter all-reduce, max over ranks,
barrier) on the GPU box with ONE rank: RCCL refuses two ranks on one GPU, and
the driver's multi-GPU run is the only N>1 test.  Launch:
  python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 tools/nccl_rehearsal.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402

local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))  # as bench.dist_setup
ctr = np.arange(14, dtype=np.int64).reshape(2, 7)
out = bench.allreduce_counters(dist, ctr, local)
assert np.array_equal(out, ctr * dist.get_world_size()), out
assert bench.max_over_ranks(dist, 1.5, local) == 1.5
bench.barrier(dist, local)
print("rccl path ok: world", dist.get_world_size(), "backend", dist.get_backend(), flush=True)
dist.destroy_process_group()
