"""VALU list scheduling for the generated gfx950 kernels (bs_codegen IR).

tools/ubench_dep.hip (profiles/r05_ubench_dep.json) measures a dependent
v_xor / v_bitop3 at about 8-9 cycles issue to issue, against 4 cycles for
independent instructions of one wave: with two waves per SIMD a stream whose
every op consumes the previous one's result issues at 0.54 per SIMD per ns,
two interleaved chains 0.70, four 0.88, eight 0.96.  The generators emit the
work in program order (a transpose's shift right before the selects that use
it, a product right before its accumulate); this pass reorders each run of
plain VALU ops between two non-VALU ops (loads, stores, waits, exec and SALU
changes, labels, branches stay where they are, and so does everything
relative to them) so that an op's producers sit at least LAT ops earlier
where the run allows it, keeping every true, anti and output dependency.

Only ops whose register reads and writes are known here are moved; any other
op ends the run.  The emulator runs the scheduled kernels in every CPU test
that goes through bs_codegen.generate (a reordering that broke a dependency
would change their results).
"""
from __future__ import annotations

from typing import Optional

LAT = 2   # issue slots between a producer and its first consumer (one wave: ~8 of 4-cycle slots)


def _rw(op) -> Optional[tuple[set, set]]:
    """(registers written, registers read) of a schedulable VALU op, or None."""
    n, a = op.name, op.args
    if n in ("v_xor", "v_sub"):
        return {a[0]}, {a[1], a[2]}
    if n == "v_mov":
        return {a[0]}, {a[1]}
    if n == "v_xor3":
        return {a[0]}, {a[1], a[2], a[3]}
    if n == "v_bitsel_s":
        return {a[0]}, {a[2], a[3]}
    if n == "v_bitsel_v":
        return {a[0]}, {a[1], a[2], a[3]}
    if n == "v_movk":
        return {a[0]}, set()
    if n in ("v_andk", "v_lshr", "v_lshl", "v_addk"):
        return {a[0]}, {a[2]}
    if n in ("v_lshl64", "v_lshr64"):
        return {a[0], a[0] + 1}, {a[2], a[2] + 1}
    if n == "v_perm":
        return {a[0]}, {a[1], a[2], a[3]}
    if n == "v_perm_s":
        return {a[0]}, {a[1], a[2]}
    return None


def _schedule_run(run: list, lat: int = LAT) -> list:
    """List-schedule one run of (op, writes, reads): greedy, earliest original
    position first among the ops whose producers issued >= LAT slots ago."""
    n = len(run)
    if n < 3:
        return [op for op, _, _ in run]
    preds = [set() for _ in range(n)]
    last_w: dict = {}
    reads_since: dict = {}
    for i, (_, w, r) in enumerate(run):
        for x in r:                       # true dependencies
            if x in last_w:
                preds[i].add(last_w[x])
        for x in w:                       # output and anti dependencies
            if x in last_w:
                preds[i].add(last_w[x])
            for j in reads_since.get(x, ()):
                if j != i:
                    preds[i].add(j)
        for x in r:
            reads_since.setdefault(x, []).append(i)
        for x in w:
            last_w[x] = i
            reads_since[x] = []
    true_pred = [set() for _ in range(n)]
    last_w = {}
    for i, (_, w, r) in enumerate(run):
        for x in r:
            if x in last_w:
                true_pred[i].add(last_w[x])
        for x in w:
            last_w[x] = i
    succs = [[] for _ in range(n)]
    npred = [len(p) for p in preds]
    for i, p in enumerate(preds):
        for j in p:
            succs[j].append(i)
    issued_at = [-1] * n
    ready = sorted(i for i in range(n) if npred[i] == 0)
    out, t = [], 0
    while ready:
        pick = None
        for i in ready:
            if all(t - issued_at[j] >= lat for j in true_pred[i]):
                pick = i
                break
        if pick is None:
            pick = ready[0]
        ready.remove(pick)
        issued_at[pick] = t
        t += 1
        out.append(run[pick][0])
        for s in succs[pick]:
            npred[s] -= 1
            if npred[s] == 0:
                # keep the ready list in original order
                lo, hi = 0, len(ready)
                while lo < hi:
                    mid = (lo + hi) // 2
                    if ready[mid] < s:
                        lo = mid + 1
                    else:
                        hi = mid
                ready.insert(lo, s)
    assert len(out) == n
    return out


def schedule(ops: list, lat: int = LAT) -> list:
    """The kernel's op list with every run of schedulable VALU ops reordered."""
    out, run = [], []
    for op in ops:
        rw = _rw(op)
        if rw is None:
            out.extend(_schedule_run(run, lat))
            run = []
            out.append(op)
        else:
            run.append((op,) + rw)
    out.extend(_schedule_run(run, lat))
    return out


def stall_slots(ops: list, lat: int = LAT) -> tuple[int, int]:
    """(schedulable VALU ops, issue slots one wave needs for them in order
    with `lat` slots from producer to consumer): a static measure of the
    dependency stalls the order leaves (runs are bounded as in schedule)."""
    n_ops = slots = 0
    t = 0
    ready_at: dict = {}
    for op in ops:
        rw = _rw(op)
        if rw is None:
            ready_at = {}
            continue
        w, r = rw
        start = max([t] + [ready_at.get(x, 0) for x in r])
        t = start + 1
        for x in w:
            ready_at[x] = start + lat
        n_ops += 1
    slots = t
    return n_ops, slots
