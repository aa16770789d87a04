#!/usr/bin/env python3
"""Summarise FFTCONV_LA_TRACE launch timelines (csrc/la.hpp upols_la_kernel):
per role (0 level-3 anchor, 1 level-2 anchor, 2 step, 3 level-1 anchor, 4 mix
walk; csrc/la.hpp la_role) when its waves start
and end, relative to the launch's first wave (s_memrealtime ticks, 10 ns)."""
import sys

import numpy as np

ROLES = {0: "level3", 1: "level2", 2: "step", 3: "level1", 4: "mixwalk", 5: "pad", 6: "proc"}


def load(path):
    raw = open(path, "rb").read()
    slots, grid, C, B = np.frombuffer(raw[:32], np.int64)
    meta = np.frombuffer(raw[32:32 + 16 * slots], np.int64).reshape(slots, 2)
    allr = np.frombuffer(raw[32 + 16 * slots:], np.int32).reshape(slots, 2, grid, 4, 4)
    return int(C), int(B), meta, allr[:, 0], allr[:, 1]


def summarise(path):
    C, B, meta, rec, stamps = load(path)
    ph = {}
    lines = []
    spans = []
    per_role = {}
    for s in range(rec.shape[0]):
        if meta[s, 0] < 0:
            continue
        r = rec[s].reshape(-1, 4)
        st = stamps[s].reshape(-1, 4).astype(np.int64) & 0xffffffff
        keep = (r[:, 2] != 0) | (r[:, 3] != 0)
        r, st = r[keep], st[keep]
        if len(r) == 0:
            continue
        t0 = r[:, 2].astype(np.int64) & 0xffffffff
        t1 = r[:, 3].astype(np.int64) & 0xffffffff
        base = t0.min()
        t0 -= base
        t1 -= base
        spans.append(t1.max())
        role = r[:, 0] & 15
        wave = (r[:, 0] >> 4) & 15
        for k in np.unique(role):
            for w in (0, 2):  # chain wave / helper wave of the step role
                nchain = 1 if k == 6 else 2  # (process launch: wave 0 is the chain)
                m = (role == k) & ((wave >= nchain) == (w == 2))
                for q in range(4):
                    mm = m & (st[:, q] != 0)
                    if mm.any():  # (relative to each wave's own start: a run's last call)
                        own = r[mm, 2].astype(np.int64) & 0xffffffff
                        ph.setdefault((int(k), w, q), []).append(np.median(st[mm, q] - own))
            m = role == k
            d = per_role.setdefault(int(k), {"n": [], "start": [], "end": [], "dur": []})
            d["n"].append(int(m.sum()))
            d["start"].append(np.percentile(t0[m], [0, 50, 100]))
            d["end"].append(np.percentile(t1[m], [0, 50, 90, 100]))
            d["dur"].append(np.percentile((t1 - t0)[m], [50, 90, 100]))
    lines.append(f"{path}: C={C} B={B}, {len(spans)} launches, span median {np.median(spans) / 100:.2f} us "
                 f"(min {np.min(spans) / 100:.2f}, max {np.max(spans) / 100:.2f})")
    for k, d in sorted(per_role.items()):
        st = np.median(np.array(d["start"]), axis=0) / 100
        en = np.median(np.array(d["end"]), axis=0) / 100
        du = np.median(np.array(d["dur"]), axis=0) / 100
        lines.append(f"  {ROLES.get(k, k):8s} waves/launch {int(np.median(d['n'])):5d}  start min/med/max "
                     f"{st[0]:6.2f} {st[1]:6.2f} {st[2]:6.2f}  end min/med/p90/max {en[0]:6.2f} {en[1]:6.2f} "
                     f"{en[2]:6.2f} {en[3]:6.2f}  dur med/p90/max {du[0]:6.2f} {du[1]:6.2f} {du[2]:6.2f} us")
    for (k, w, q), v in sorted(ph.items()):
        lines.append(f"  phase stamp role {ROLES.get(k, k)} {'chain' if w == 0 else 'helper'} wave, stamp {q}: "
                     f"median {np.median(v) / 100:6.2f} us")
    return "\n".join(lines)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        try:
            print(summarise(p))
        except (ValueError, OverflowError) as e:  # (a record from a handle with no traced launches)
            print(f"{p}: unreadable record ({e})")
