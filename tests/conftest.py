import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: larger CPU oracle runs")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def engine_lib():
    import __graft_entry__ as g
    g.build_engine()
    from mops_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def small_case():
    """2.4k-cell culled mesh, 10 levels, one snapshot (+ a phase-shifted one)."""
    from mops_amd import synth
    mesh = synth.make_mesh(16, n_levels=10)
    s0 = synth.make_snapshot(mesh, timestep=0, phase=0.0)
    s1 = synth.make_snapshot(mesh, timestep=1, phase=0.35)
    return mesh, s0, s1


@pytest.fixture(scope="session")
def medium_case():
    """41k-cell mesh, 60 levels (EC30to60-like vertical grid)."""
    from mops_amd import synth
    mesh = synth.make_mesh(64, n_levels=60)
    s0 = synth.make_snapshot(mesh, timestep=0, phase=0.0)
    s1 = synth.make_snapshot(mesh, timestep=1, phase=0.35)
    return mesh, s0, s1
