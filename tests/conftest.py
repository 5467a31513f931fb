import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the gfx950 kernels)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def dfp():
    # (re)build the in-tree library if a source is newer than it (no-op otherwise)
    sys.path.insert(0, os.path.join(ROOT, "datafusion-parallelism_amd"))
    import build as hipbuild

    sys.path.pop(0)
    hipbuild.build()
    import datafusion_parallelism_amd as m

    m.load()
    return m


def init_one_rank_nccl():
    """A one-rank RCCL process group on cuda:0 whose rendezvous is an in-memory store: a
    free TCP port picked by binding port 0 and closing it can be taken again before the
    store listens on it (EADDRINUSE seen on the GPU box, gpurun_out/r05y/tests.log)."""
    import torch
    import torch.distributed as dist

    os.environ.update(RANK="0", WORLD_SIZE="1")
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=torch.device("cuda", 0))
