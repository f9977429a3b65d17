import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "gpu-ecs-madrona_amd"))

# Load the framework early (it imports torch first so both share torch's
# HIP runtime; madrona_mi355x/__init__.py explains why).
try:
    import madrona_mi355x  # noqa: F401,E402
except ImportError:
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def _build_oracle():
    """Build the oracle restatement (and the reference harness when the
    reference sources are present) once per session.  CPU-only, seconds."""
    orc = os.path.join(ROOT, "oracle", "_build", "liborc.so")
    if not os.path.exists(orc) or os.environ.get("MW_REBUILD_ORACLE"):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    yield


def pytest_assertrepr_compare(config, op, left, right):
    """A failed `a.tobytes() == b.tobytes()` on large buffers: report the
    lengths and the first differing byte instead of pytest's difflib
    explanation, which is quadratic and takes minutes on megabyte buffers
    (long enough for a GPU box to take the run for hung)."""
    if op == "==" and isinstance(left, (bytes, bytearray)) and isinstance(right, (bytes, bytearray)):
        n = min(len(left), len(right))
        first = next((i for i in range(n) if left[i] != right[i]), n)
        return [f"byte buffers differ: len {len(left)} vs {len(right)}, first difference at byte {first}"]
    return None
