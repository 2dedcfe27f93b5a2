import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rte-rrtmgp-nn_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box with -m gpu)")


@pytest.fixture(params=[1, 2, 3], ids=["sw1", "sw2", "sw3"])
def sw_kernel(request):
    """Force each SW two-stream kernel (one / two g-points per lane / checkpointed passes) for the test, then restore
    the size rule."""
    from rrtmgpnn import api
    api.set_sw_kernel_default(request.param)
    yield request.param
    api.set_sw_kernel_default(0)


@pytest.fixture(params=[0, 1], ids=["mlp32", "mlp16"])
def mlp_kernel(request):
    """Force each MFMA tiling of the gas-optics networks (32x32x2 where instantiated / 16x16x4) for the test, then restore
    the default."""
    from rrtmgpnn import api
    api.set_mlp_kernel_default(request.param)
    yield request.param
    api.set_mlp_kernel_default(0)


@pytest.fixture(scope="session")
def orc():
    import oracle as O
    return O.Oracle()


@pytest.fixture(scope="session")
def rfmip():
    from rrtmgpnn import data
    return data.rfmip_problem()


def subset(prob, idx):
    import numpy as np
    idx = np.asarray(idx)
    sub = {k: (v[idx] if isinstance(v, np.ndarray) and v.ndim >= 1 and v.shape[0] == prob["ncol"] else v)
           for k, v in prob.items()}
    sub["gases"] = {k: v[idx] for k, v in prob["gases"].items()}
    sub["ncol"] = len(idx)
    return sub
