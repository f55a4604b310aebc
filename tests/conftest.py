"""pytest configuration: markers, import helpers and shared fixtures.

`-m gpu` tests run on a real MI355X (they call the HIP library through its C-ABI and compare with
the oracle); everything else is CPU-only (oracle vs golden fixtures, host codec, ABI exports).
"""
import contextlib
import importlib
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
ORACLE_DIR = os.path.join(REPO, "oracle")
if ORACLE_DIR not in sys.path:
    sys.path.insert(0, ORACLE_DIR)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def pkg():
    return importlib.import_module("3ddctvideoencoding_amd")


@pytest.fixture(scope="session")
def oracle():
    import oracle as o  # oracle/oracle.py (test infrastructure)
    return o


@pytest.fixture(scope="session")
def plan8(oracle):
    return oracle.Plan(8, 8, 8)


@pytest.fixture(scope="session")
def plan4(oracle):
    return oracle.Plan(8, 8, 4)


@contextlib.contextmanager
def ctx_option(ctx, option, value):
    """Set a test / diagnostic option (DCT3D_OPT_*) on a context for the duration of a block."""
    ctx.set_option(option, value)
    try:
        yield ctx
    finally:
        ctx.set_option(option, 0)


@pytest.fixture(scope="session")
def gpu_ctx8(pkg):
    try:
        ctx = pkg.Context(0, 8, 8, 8)
    except Exception as e:  # on the GPU box a missing device / library is a failure, not a skip
        pytest.fail(f"HIP context for 8x8x8 could not be created: {e}")
    yield ctx
    ctx.close()


@pytest.fixture(scope="session")
def gpu_ctx4(pkg):
    try:
        ctx = pkg.Context(0, 8, 8, 4)
    except Exception as e:
        pytest.fail(f"HIP context for 8x8x4 could not be created: {e}")
    yield ctx
    ctx.close()
