import json
import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def load_golden(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """GPU runs: torch's HIP runtime starts before the library's, as in bench.py.  torch ships its own
    HIP / HSA runtime; with the library's already up, torch found no device (tests/test_gpu_dist.py run
    after tests/test_gpu_edge.py), while this order serves both (the -m gpu suite, bench.py)."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass
    yield


@pytest.fixture
def heartbeat(request):
    """For tests that run for minutes in one call (the per-GPU-share scale tests): a progress line on the
    process's real stderr every 30 s (pytest captures the test's own output until it ends), so a
    watchdog that takes a silent command for a hung one sees it working."""
    import threading
    import time
    stop = threading.Event()
    t0 = time.time()
    name = request.node.name

    # fd-level capture holds fd 2 too: the line is written with capture suspended, and appended to
    # gpurun_out/heartbeat.log when that directory exists (the GPU box's watchdog reads both)
    capman = request.config.pluginmanager.getplugin("capturemanager")
    root = os.environ.get("GRAFT_REPO_ROOT")
    hb_file = os.path.join(root, "gpurun_out", "heartbeat.log") if root else None

    def beat():
        while not stop.wait(30.0):
            line = f"[heartbeat] {name}: {time.time() - t0:.0f}s\n"
            try:
                if capman is not None:
                    with capman.global_and_fixture_disabled():
                        sys.stderr.write(line)
                        sys.stderr.flush()
                else:
                    sys.__stderr__.write(line)
                    sys.__stderr__.flush()
            except Exception:
                pass
            if hb_file and os.path.isdir(os.path.dirname(hb_file)):
                try:
                    with open(hb_file, "a") as f:
                        f.write(line)
                except OSError:
                    pass

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()
    th.join(timeout=5)
