"""Every cross-stream handoff in the engine carries the ordering tests' spin hook.

tests/test_gpu_ordering.py makes a missing wait fail deterministically by queueing a spin kernel on
a stream after each of its cross-stream waits (so what it produces next starts late) and before
each event another stream or host thread waits on (the test hook "handoff_spin",
include/scde_hip.h).  That only covers the handoffs that call the hook, so this check reads
engine.hip: each `hipEventRecord` is either one of the profiling marks (timing events of one
stream, never waited on by another) or is immediately preceded by a `handoff_spin(...)` on the
same stream, and every `hipStreamWaitEvent` sits inside `handoff_wait`, which spins after the
wait.  A new handoff added without the hook fails here.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENGINE = os.path.join(ROOT, "scde_amd", "csrc", "engine.hip")


def _records(lines):
    for i, line in enumerate(lines):
        m = re.search(r"hipEventRecord\(([^,]+),\s*([^)]+)\)", line)
        if m:
            yield i, m.group(1).strip(), m.group(2).strip()


def test_every_cross_stream_event_is_preceded_by_the_spin_hook():
    lines = open(ENGINE).read().split("\n")
    recs = list(_records(lines))
    assert len(recs) >= 14, recs  # the pipelined host path's handoffs (and the two timing marks)
    missing = []
    for i, ev, stream in recs:
        if ev in ("a", "b") and "(void)" in lines[i]:  # mark_begin / mark_end timing events
            continue
        prev = lines[i - 1]
        m = re.search(r"handoff_spin\(([^,]+),\s*([^)]+)\)", prev)
        if not m or m.group(2).strip() != stream:
            missing.append(f"engine.hip:{i + 1}: hipEventRecord({ev}, {stream}) without handoff_spin on {stream}")
    assert not missing, "\n".join(missing)


def test_every_cross_stream_wait_goes_through_handoff_wait():
    src = open(ENGINE).read()
    m = re.search(r"static hipError_t handoff_wait\([^)]*\)\s*\{(.*?)\n\}", src, re.S)
    assert m, "handoff_wait helper missing"
    body = m.group(1)
    assert "hipStreamWaitEvent" in body and "handoff_spin" in body
    assert body.index("hipStreamWaitEvent") < body.index("handoff_spin")  # spin after the wait
    rest = src[: m.start()] + src[m.end():]
    raw = [f"engine.hip:{src[: src.index(l)].count(chr(10)) + 1}: {l.strip()}"
           for l in rest.split("\n") if "hipStreamWaitEvent(" in l]
    assert not raw, "raw waits outside handoff_wait:\n" + "\n".join(raw)
    assert src.count("handoff_wait(") + src.count("lane_join(") >= 16


def test_spin_hook_is_reachable_from_the_api():
    src = open(ENGINE).read()
    assert '"handoff_spin"' in src and "spin_cycles" in src and '"skip_lane_join"' in src
    hdr = open(os.path.join(ROOT, "include", "scde_hip.h")).read()
    assert "handoff_spin" in hdr and "scde_ctx_inject_fault" in hdr
