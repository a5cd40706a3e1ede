"""The asm look-ahead in k_boot2 and k_boot_tiles (column loads issued from inline asm and
waited with an explicit vmcnt) is only correct while the compiler keeps the loaded registers
in place between the asm load and its wait: a spill or register copy in between reads the
register before the data lands, or reuses it while the load is still in flight.  Builds that
spill inside those loops have faulted on the GPU.  This test compiles
kernels.hip for gfx950 (device only, as the library is built) and checks that no loop of those
kernels (and of k_boot2_list, whose item loop holds k_boot2's body) touches scratch memory.
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "scde_amd", "csrc")


@pytest.fixture(scope="module")
def isa(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not found")
    out = tmp_path_factory.mktemp("isa") / "kernels.s"
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--cuda-device-only",
                        "-S", "-I" + os.path.join(ROOT, "include"), "-o", str(out), os.path.join(CSRC, "kernels.hip")],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    return out.read_text()


def _bodies(isa, name_re):
    """(symbol, body text) of every kernel whose mangled name matches name_re."""
    out = []
    for m in re.finditer(r"^(_ZN4scde[^\s:]*" + name_re + r"[^\s:]*):", isa, re.M):
        start = m.end()
        end = isa.find(".Lfunc_end", start)
        out.append((m.group(1), isa[start:end]))
    return out


def _loop_spans(body):
    """Line spans [header, last back-branch] of the loops in a kernel body."""
    lines = body.split("\n")
    labels = {}
    for i, ln in enumerate(lines):
        m = re.match(r"^(\.LBB\d+_\d+):", ln)
        if m:
            labels[m.group(1)] = i
    spans = []
    for i, ln in enumerate(lines):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", ln)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i and "Loop Header" in "\n".join(lines[labels[tgt]:labels[tgt] + 2]):
                spans.append((labels[tgt], i))
    return lines, spans


@pytest.mark.parametrize("kernel", ["k_boot2ILi20E", "k_boot_tilesILi20E", "k_boot2_listILi20E"])
def test_lookahead_loops_do_not_touch_scratch(isa, kernel):
    bodies = _bodies(isa, kernel)
    assert bodies, f"{kernel} not found in the ISA"
    for sym, body in bodies:
        lines, spans = _loop_spans(body)
        assert spans, f"no loops found in {sym}"
        for a, b in spans:
            bad = [ln.strip() for ln in lines[a:b + 1] if "scratch_" in ln or "buffer_store" in ln]
            assert not bad, f"{sym}: scratch access inside a loop: {bad[:3]}"


def test_tables_register_row_does_not_spill(isa):
    """k_tables_reg keeps a column's 401 grid values in VGPRs; builds that spilled them (or
    the hoisted polynomial constants) to scratch ran 15-40 % slower."""
    bodies = _bodies(isa, "k_tables_reg")
    assert len(bodies) == 6, [s for s, _ in bodies]
    for sym, body in bodies:
        bad = [ln.strip() for ln in body.split("\n") if "scratch_" in ln]
        assert not bad, f"{sym}: scratch access: {bad[:3]}"
