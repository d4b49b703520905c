import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # tests are allowed to load the oracle


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def gpu_available() -> bool:
    try:
        import pathtracerwithcuda_amd as pt
        return pt.device_count() > 0
    except Exception:
        return False


@pytest.hookimpl(hookwrapper=True)
def pytest_runtest_makereport(item, call):
    """A test that needs the reference's own assets (bench.asset_root: tests/golden/ref_assets.tar.xz, generated from
    a reference checkout and kept out of git) is skipped where the pack is absent."""
    outcome = yield
    rep = outcome.get_result()
    if call.excinfo is not None and call.excinfo.typename == "ReferenceAssetsMissing":
        rep.outcome = "skipped"
        rep.longrepr = (str(item.fspath), item.location[1] or 0, f"Skipped: {call.excinfo.value}")


@pytest.fixture(scope="session")
def require_gpu():
    if not gpu_available():
        pytest.fail("no HIP device visible: the -m gpu tests must run on the MI355X box")
