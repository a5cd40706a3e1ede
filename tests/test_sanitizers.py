"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 sanitizers row).

Two builds (``make sanitize`` in scde_amd/csrc and oracle/, outputs under build/asan/):

* the library's host code (hipcc with the sanitizers after -Xarch_host: device code is
  unchanged), loaded alone (no torch) in a child process under clang's ASan runtime: BH / cZ
  on the host, R's Mersenne-Twister and sample(), the set_random_matrices shuffles, the
  layer-1 argument checks and the no-GPU error paths;
* the oracle (gcc -fsanitize=address,undefined), under gcc's runtime: the whole
  scde.expression.difference restatement (tables, bootstrap, ratio, summary, BH), the batch
  branch, the weighted PCA and the PAGODA helpers.

Each child exits non-zero on the first sanitizer report (halt_on_error, no recovery).
"""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT

ASAN_DIR = os.path.join(ROOT, "build", "asan")

LIB_SCRIPT = r"""
import ctypes, numpy as np
from scde_amd import _lib, api
L = _lib.lib()
rng = np.random.default_rng(5)
z = rng.normal(0, 3, 4001); z[::17] = np.nan; z[3] = 0.0
cz = api.bh_cz(z)
assert np.isnan(cz[0]) and np.all(np.isfinite(cz[1:][~np.isnan(z[1:])]))
from scde_amd import pagoda as PG
st = PG.RState(42)
u = st.unif_rand(3000); s = st.sample(500, 200)
assert u.min() > 0 and u.max() < 1 and len(set(s.tolist())) == 200
p = PG.shuffle_perms(7, 2, 5, 300)
assert sorted(p.reshape(-1, 300)[3].tolist()) == list(range(300))
h = ctypes.c_void_p()
assert L.scde_ctx_create(0, ctypes.byref(h)) != 0        # no GPU in this process: a clean error
try:                                                     # shape errors are reported, not UB
    api.logBootPosterior(np.zeros((3, 12)), [np.array([0]), np.array([0]), np.array([0])], np.full((2, 3), 5), np.zeros(4), 10, 1)
    raise SystemExit("expected an error")
except api.ScdeError:
    pass
print("library host paths clean")
"""

ORACLE_SCRIPT = r"""
import numpy as np
from conftest import golden
from oracle import oracle as O, wpca as W, pagoda as OP
g = golden("esmef500.npz")
models = {c: g["models"][:, j] for j, c in enumerate(O.MODEL_COLUMNS) if not np.all(np.isnan(g["models"][:, j]))}
counts = np.ascontiguousarray(g["counts"][:40])
r = O.scde_expression_difference(models, counts, g["prior_x"], g["prior_y"], g["groups"], n_randomizations=8, n_cores=3,
                                 return_posteriors=True)
assert np.all(np.isfinite(r["results"]["Z"]))
batch = np.array([i % 2 for i in range(counts.shape[1])])
O.scde_expression_difference_batch(models, counts, g["prior_x"], g["prior_y"], g["groups"], batch, n_randomizations=5,
                                   n_cores=2)
O.scde_posteriors(models, counts, g["prior_x"], n_randomizations=5, return_individual_posteriors=True,
                  return_individual_posterior_modes=True, n_cores=1)
rng = np.random.default_rng(1)
m = rng.normal(size=(60, 12)); w = rng.uniform(0.1, 1, size=(60, 12))
W.baileyWPCA(m, w, 2, 2, 0, 1e-6, 10, W.RState(3).unif_rand(2 * 12 * 2), 0, None)
OP.winsorizeMatrix(rng.normal(size=(7, 30)), 0.1)
OP.matWCorr(m, w)
print("oracle clean")
"""


def _run(script, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    env["PYTHONPATH"] = os.pathsep.join([ROOT, os.path.join(ROOT, "tests")])
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    return subprocess.run([sys.executable, "-c", script], env=env, capture_output=True, text=True, timeout=600,
                          cwd=ROOT)


def _ensure(target, path):
    if not os.path.exists(path):
        d = os.path.join(ROOT, "scde_amd", "csrc") if "scde_hip" in path else os.path.join(ROOT, "oracle")
        if subprocess.run(["make", "-s", "-j8", "-C", d, "sanitize"], capture_output=True).returncode != 0:
            pytest.skip(f"{target}: sanitizer build failed")
    nm = shutil.which("nm")
    if nm:  # the build really is instrumented: it calls the ASan and UBSan report hooks
        syms = subprocess.run([nm, "-D", path], capture_output=True, text=True).stdout
        assert "__asan_report" in syms and "__ubsan_handle" in syms, f"{path} is not instrumented"
    return path


def test_library_host_code_under_asan_ubsan():
    lib = _ensure("library", os.path.join(ASAN_DIR, "libscde_hip_asan.so"))
    rt = None
    for root, _, files in os.walk("/opt/rocm/lib/llvm/lib/clang"):
        if "libclang_rt.asan-x86_64.so" in files:
            rt = os.path.join(root, "libclang_rt.asan-x86_64.so")
    if rt is None:
        pytest.skip("clang ASan runtime not found")
    r = _run(LIB_SCRIPT, {"LD_PRELOAD": rt, "SCDE_LIB": lib, "SCDE_SKIP_TORCH": "1"})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "library host paths clean" in r.stdout


def test_oracle_under_asan_ubsan():
    lib = _ensure("oracle", os.path.join(ASAN_DIR, "liboracle.so"))
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("gcc not found")
    asan = subprocess.run([gcc, "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    r = _run(ORACLE_SCRIPT, {"LD_PRELOAD": asan, "SCDE_ORACLE_LIB": lib})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "oracle clean" in r.stdout
