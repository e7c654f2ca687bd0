"""The JavaScript host path: N-API addon + streams-api.mjs (zlib-streams-ts_amd/js)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = os.path.join(ROOT, "zlib-streams-ts_amd", "js")
ADDON = os.path.join(JS, "zsnapi.node")

need_node = pytest.mark.skipif(shutil.which("node") is None or not os.path.exists(ADDON),
                               reason="node or the built addon (make -C zlib-streams-ts_amd/js) is missing")


@need_node
def test_addon_loads_and_fails_loudly_without_gpu():
    env = dict(os.environ)
    try:
        import torch
        if torch.cuda.is_available():
            env["ZS_EXPECT_GPU"] = "1"
    except ImportError:
        pass
    r = subprocess.run(["node", os.path.join(JS, "test", "load.test.mjs")], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


@need_node
@pytest.mark.gpu
def test_js_batch_api_matches_reference_goldens():
    r = subprocess.run(["node", os.path.join(JS, "test", "batch.test.mjs")], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ")
