import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


def _load(name, path):
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def oracle():
    """CPU oracle (test infrastructure only)."""
    return _load("sgm_oracle", os.path.join(ROOT, "oracle", "sgm_oracle.py"))


@pytest.fixture(scope="session")
def synth():
    return _load("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))


@pytest.fixture(scope="session")
def pkg():
    return ge.load_package()


@pytest.fixture(scope="session")
def engine(pkg):
    if pkg.device_count() < 1:
        pytest.fail("no HIP device visible — GPU tests must run on the MI355X box")
    eng = pkg.Engine(0)
    yield eng
    eng.close()


def to_oracle_params(oracle, p):
    d = p.as_dict()
    mode = d.pop("mode")
    return oracle.make_params(mode, **d)
