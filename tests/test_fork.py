"""Fork safety (threading row): R's mclapply forks worker processes after
the package's library is loaded, and each worker makes its own .Call.  Loading
libscde_hip.so must therefore not touch HIP: a context (and the HIP runtime behind it) is
created lazily, on the first call in the process that makes it.

The test runs a fresh interpreter (the pytest process itself has used the GPU, and a
process that has must not fork into GPU work): it loads the library, calls a host-only
entry (the BH adjustment), forks, lets the child run scde.expression.difference on the GPU
as an mclapply worker would, then runs the same call in the parent after the child has
exited; both tables must be identical.
"""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import os, sys
    import numpy as np
    sys.path.insert(0, {root!r})
    from scde_amd import api
    g = np.load(os.path.join({root!r}, "tests", "golden", "esmef500.npz"), allow_pickle=False)
    from oracle.oracle import MODEL_COLUMNS
    models = {{c: g["models"][:, j] for j, c in enumerate(MODEL_COLUMNS) if not np.all(np.isnan(g["models"][:, j]))}}
    counts = np.ascontiguousarray(g["counts"][:48])
    prior = {{"x": g["prior_x"], "y": g["prior_y"]}}
    groups = list(g["groups"])
    # the library is loaded and a host-only entry has run: no HIP context may exist yet
    cz = api.bh_cz(np.array([1.0, -2.0, 3.0]))
    assert np.all(np.isfinite(cz))

    def table():
        api.set_rand("glibc")
        r = api.scde_expression_difference(models, counts, prior, groups=groups, n_randomizations=10, n_cores=2)
        return np.column_stack([r[k].to_numpy() for k in ("lb", "mle", "ub", "ce", "Z", "cZ")])

    out = sys.argv[1]
    pid = os.fork()
    if pid == 0:  # the worker: its first HIP use happens after the fork
        try:
            np.save(out, table())
            code = 0
        except BaseException as e:  # noqa: BLE001
            print("child failed:", repr(e), flush=True)
            code = 1
        os._exit(code)
    _, status = os.waitpid(pid, 0)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, status
    child = np.load(out + ".npy")
    parent = table()
    assert np.array_equal(child, parent, equal_nan=True), (child[:3], parent[:3])
    print("fork ok", child.shape)
""")


SCRIPT_AFTER_INIT = textwrap.dedent("""
    import ctypes, os, sys
    import numpy as np
    sys.path.insert(0, {root!r})
    from scde_amd import api, _lib
    g = np.load(os.path.join({root!r}, "tests", "golden", "esmef500.npz"), allow_pickle=False)
    from oracle.oracle import MODEL_COLUMNS
    models = {{c: g["models"][:, j] for j, c in enumerate(MODEL_COLUMNS) if not np.all(np.isnan(g["models"][:, j]))}}
    counts = np.ascontiguousarray(g["counts"][:48])
    prior = {{"x": g["prior_x"], "y": g["prior_y"]}}
    groups = list(g["groups"])

    def table():
        api.set_rand("glibc")
        r = api.scde_expression_difference(models, counts, prior, groups=groups, n_randomizations=10, n_cores=1)
        return np.column_stack([r[k].to_numpy() for k in ("lb", "mle", "ub", "ce", "Z", "cZ")])

    first = table()  # the parent initialises HIP (R: an n.cores = 1 call in the session)
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:  # an mclapply worker forked after that: its GPU call must fail cleanly
        os.close(r)
        msg = "no error"
        try:
            table()
        except _lib.ScdeError as e:
            msg = "ScdeError " + str(e)
        except BaseException as e:  # noqa: BLE001
            msg = "other " + repr(e)
        L = _lib.lib()
        h = ctypes.c_void_p()
        rc = L.scde_ctx_create(0, ctypes.byref(h))
        msg += " | ctx_create rc=%d" % rc
        os.write(w, msg.encode())
        os.close(w)
        os._exit(0)  # no destructors, no HIP call in the child
    os.close(w)
    child = b""
    while True:
        chunk = os.read(r, 4096)
        if not chunk:
            break
        child += chunk
    _, status = os.waitpid(pid, 0)
    child = child.decode()
    print("child:", child)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, status
    assert child.startswith("ScdeError scde_hip error 4:") and "forked" in child, child
    assert child.endswith("ctx_create rc=4"), child
    again = table()  # the parent's runtime is untouched
    assert np.array_equal(first, again, equal_nan=True)
    print("fork-after-init ok")
""")


@pytest.mark.gpu
def test_fork_after_init_child_gets_error(tmp_path):
    """SURVEY.md §8(b) threading row (VERDICT r03 missing #3): the parent initialises HIP,
    forks; the child's GPU entries return SCDE_EFORK before any HIP call and the child _exits;
    the parent's next call still works and gives the same table."""
    script = tmp_path / "fork_after_init.py"
    script.write_text(SCRIPT_AFTER_INIT.format(root=ROOT))
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "fork-after-init ok" in r.stdout


@pytest.mark.gpu
def test_fork_after_load_then_gpu_in_child_and_parent(tmp_path):
    script = tmp_path / "fork_child.py"
    script.write_text(SCRIPT.format(root=ROOT))
    r = subprocess.run([sys.executable, str(script), str(tmp_path / "child")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "fork ok" in r.stdout


def test_library_load_is_host_only():
    """On a machine without a GPU (this container) the library still loads and its host-only
    entries run: nothing at load time needs the HIP runtime's devices."""
    code = ("import sys, numpy as np; sys.path.insert(0, %r); from scde_amd import api; "
            "print(api.bh_cz(np.array([0.5, -1.5])).tolist())" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
