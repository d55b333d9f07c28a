"""RCCL (torch.distributed backend "nccl") on the real device: the process
group the 8-GPU data-parallel bench joins, rehearsed as the single rank of
a world of one (a one-GPU box cannot host two RCCL ranks).  Exercises
`cadence.distributed.init_from_env` with `device_id`, the one
`all_gather_into_tensor` of `gather_rows`, `max_over_ranks` and the barrier,
with HSA_ENABLE_IPC_MODE_LEGACY=0 as on the node.  Runs in a
child process so the process group never leaks into other tests."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import torch, torch.distributed as dist
from cadence import distributed as D
rank, world, local = D.init_from_env()
assert (rank, world, local) == (0, 1, 0), (rank, world, local)
assert dist.is_initialized() and dist.get_backend() == "nccl", dist.get_backend()
x = torch.arange(24, dtype=torch.int32, device="cuda").view(6, 4)
y = D.gather_rows(x)
torch.cuda.synchronize()
assert torch.equal(y, x), y
assert D.max_over_ranks(2.5) == 2.5
D.barrier()
D.shutdown()
print("rccl world-1 ok", flush=True)
"""


def _free_port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


@pytest.mark.gpu
def test_rccl_world_of_one(dev):
  env = dict(os.environ, CADENCE_DIST_FORCE="1", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
             MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
             HSA_ENABLE_IPC_MODE_LEGACY="0",
             PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "cadence-gemma_amd"), ROOT,
                                         os.environ.get("PYTHONPATH", "")]))
  r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                     timeout=100)
  assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
  assert "rccl world-1 ok" in r.stdout
