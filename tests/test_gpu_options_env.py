"""SCDE_OPTIONS (include/scde_hip.h, scde_ctx_create): context options from the environment,
applied as each context is created -- the route R sessions have to the tuning options
(INTEGRATION.md).  Each case runs in a child process, since the variable is read at creation."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SCRIPT = r"""
import sys
sys.path.insert(0, {root!r})
from scde_amd import api
try:
    ctx = api.Context(0)
except Exception as e:
    print("CREATE-FAILED", e)
    sys.exit(0)
print("CREATED")
"""


def _run(env_value):
    env = dict(os.environ)
    env["SCDE_OPTIONS"] = env_value
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(root=ROOT)], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def test_known_options_apply():
    assert "CREATED" in _run("lanes=1,boot_tiles_cells=300")


def test_unknown_option_fails_creation_with_its_name():
    out = _run("lanes=1,no_such_option=3")
    assert "CREATE-FAILED" in out and "no_such_option" in out, out


def test_malformed_item_fails_creation():
    out = _run("lanes")
    assert "CREATE-FAILED" in out and "name=value" in out, out


@pytest.mark.parametrize("bad", ["lanes=abc", "boot_tiles_cells=", "lanes=2x"])
def test_non_numeric_value_fails_creation(bad):
    out = _run(bad)
    assert "CREATE-FAILED" in out and "not a number" in out, out
