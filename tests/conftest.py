import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.build()
    return O


@pytest.fixture(scope="session")
def custom_model():
    from panda_gym_amd import abi
    from panda_gym_amd.model import load_model

    return abi.make_model(load_model("panda_custom0"), ee_link=11)


@pytest.fixture(scope="session")
def upstream_model():
    from panda_gym_amd import abi
    from panda_gym_amd.model import load_model

    return abi.make_model(load_model("panda_upstream"), ee_link=6)


@pytest.fixture(params=[16, 1], ids=["wide", "narrow"])
def lanes(request):
    """Both step-kernel layouts (PandaVecEnv(lanes_per_env=...)): 16 lanes per env, 1 lane per env."""
    return request.param
