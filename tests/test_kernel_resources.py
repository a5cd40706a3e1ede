"""The asm look-ahead in k_boot2 and k_boot_tiles (column and multiplicity loads issued from
inline asm and waited with an explicit vmcnt) is only correct while the compiler keeps the
loaded registers in place between the asm load and its wait: a spill or register copy in
between reads the register before the data lands, or reuses it while the load is still in
flight.  Builds that spilled inside those loops faulted on the GPU.  This test
compiles kernels.hip for gfx950 (device only, as the library is built) and checks the loops of
those kernels (and of k_boot2_list, whose item loop holds k_boot2's body):

* no scratch traffic;
* in-flight loads (``vmcnt_hazards``): the loop body is replayed twice in program order with
  the queue of outstanding vector-memory operations (they retire in order; ``s_waitcnt
  vmcnt(N)`` leaves the N youngest in flight), and no instruction may read, write or copy a
  VGPR that an outstanding load is still to write -- the stale-read form of the same fault;
* DPP64 operands (``dpp_hazards``): a ``v_fmac_f64_dpp`` source VGPR is not written by a VALU
  instruction within the two wait states before it (k_boot_tiles' multiplicity broadcast).

``test_hazard_check_rejects_a_faulting_build`` shows the check catches the builds that faulted
(k_boot_tiles at 6 waves per SIMD).
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


_VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
_VMEM = ("global_", "buffer_", "scratch_", "flat_")


def _vregs(text):
    """VGPR numbers named in an operand string."""
    out = set()
    for m in _VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def _instructions(lines):
    """(mnemonic, operand text, from inline asm) for the instruction lines of a span."""
    out, in_asm = [], False
    for ln in lines:
        t = ln.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        t = t.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        mn, _, ops = t.partition(" ")
        out.append((mn, ops.strip(), in_asm))
    return out


def vmcnt_hazards(lines):
    """Replay a loop body twice; report instructions touching a VGPR an in-flight load writes."""
    insts = _instructions(lines)
    queue, bad = [], []
    for rep in range(2):
        for mn, ops, asm in insts:
            if mn == "s_waitcnt":
                m = re.search(r"vmcnt\((\d+)\)", ops)
                if m:
                    del queue[:max(0, len(queue) - int(m.group(1)))]
                continue
            regs = _vregs(ops)
            pending = set().union(*(d for d, _ in queue)) if queue else set()
            if mn.startswith(_VMEM):
                dst = set()
                if "load" in mn and "_lds" not in mn:  # the first operand is the destination
                    dst = _vregs(ops.split(",")[0])
                if rep == 1 and (regs & pending):
                    bad.append(f"{mn} {ops}")
                queue.append((dst, asm))
                continue
            if rep == 1 and regs & pending:
                bad.append(f"{mn} {ops}")
    return bad


def dpp_hazards(lines):
    """v_*_dpp whose src0 VGPR a VALU instruction wrote less than two wait states before."""
    insts = _instructions(lines)
    bad = []
    for i, (mn, ops, _) in enumerate(insts):
        if not mn.endswith("_dpp"):
            continue
        src0 = _vregs(ops.split(",")[1]) if "," in ops else set()
        states = 0
        for pmn, pops, _ in reversed(insts[max(0, i - 4):i]):
            if states >= 2:
                break
            if pmn == "s_nop":
                states += int(pops or 0) + 1
                continue
            if pmn.startswith("v_") and _vregs(pops.split(",")[0]) & src0:
                bad.append(f"{mn} {ops} after {pmn} {pops}")
                break
            states += 1
    return bad


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


@pytest.mark.parametrize("kernel", ["k_boot2ILi20E", "k_boot_tilesILi20E", "k_boot2_listILi20E", "k_boot_geneILi20ELi4E"])
def test_lookahead_loops_do_not_touch_scratch(isa, kernel):
    bodies = _bodies(isa, kernel)
    assert bodies, f"{kernel} not found in the ISA"
    for sym, body in bodies:
        lines, spans = _loop_spans(body)
        assert spans, f"no loops found in {sym}"
        for a, b in spans:
            bad = [ln.strip() for ln in lines[a:b + 1] if "scratch_" in ln or "buffer_store" in ln]
            assert not bad, f"{sym}: scratch access inside a loop: {bad[:3]}"


@pytest.mark.parametrize("kernel", ["k_boot2ILi20E", "k_boot_tilesILi20E", "k_boot2_listILi20E", "k_boot_geneILi20ELi4E"])
def test_lookahead_loads_not_touched_in_flight(isa, kernel):
    for sym, body in _bodies(isa, kernel):
        lines, spans = _loop_spans(body)
        for a, b in spans:
            bad = vmcnt_hazards(lines[a:b + 1])
            assert not bad, f"{sym}: VGPRs of an in-flight load touched: {bad[:3]}"


@pytest.mark.parametrize("kernel", ["k_boot_tilesILi20E", "k_boot_geneILi20ELi4E"])
def test_dpp_broadcast_sources_not_fresh_valu_results(isa, kernel):
    bodies = _bodies(isa, kernel)
    assert bodies
    for sym, body in bodies:
        assert "v_fmac_f64_dpp" in body
        bad = dpp_hazards(body.split("\n"))
        assert not bad, f"{sym}: DPP source written by VALU too recently: {bad[:3]}"


def test_hazard_check_rejects_a_faulting_build(tmp_path):
    """k_boot_tiles built for 6 waves per SIMD (the occupancy that faulted on the GPU in round 2,
    DESIGN.md §4.0), as one-wave blocks (SCDE_TILE_TEST_WB1: the shipped blocks' LDS caps
    occupancy at 4 waves per SIMD, which would leave the registers unsqueezed): the compiler
    spills or copies inside the look-ahead loop, and the check must report it."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not found")
    out = tmp_path / "k6.s"
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--cuda-device-only",
                        "-S", "-DSCDE_TILE_WPE=6", "-DSCDE_TILE_TEST_WB1", "-I" + os.path.join(ROOT, "include"),
                        "-o", str(out), os.path.join(CSRC, "kernels.hip")], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    found = []
    for sym, body in _bodies(out.read_text(), "k_boot_tilesILi20ELi1E"):
        lines, spans = _loop_spans(body)
        for a, b in spans:
            found += vmcnt_hazards(lines[a:b + 1])
            found += [ln for ln in lines[a:b + 1] if "scratch_" in ln]
    assert found, "the 6-waves-per-SIMD build shows no hazard: the check has lost its teeth"


def test_tables_lane_per_column_does_not_spill(isa):
    """k_tables_lpc (one lane per table column) keeps its running maxima,
    sums and the fallback's register row (tables_column_reg) in VGPRs; builds of the register-row
    kernel that spilled to scratch ran 15-40 % slower."""
    bodies = _bodies(isa, "k_tables_lpc")
    assert len(bodies) == 3, [s for s, _ in bodies]
    for sym, body in bodies:
        bad = [ln.strip() for ln in body.split("\n") if "scratch_" in ln]
        assert not bad, f"{sym}: scratch access: {bad[:3]}"
