"""Scenario scripts shared by the golden-fixture generator and the tests.

A scenario is a list of operations on one convolver: ("process", x, out_len)
or ("update", response).  Fixtures store them flattened:
  kind[i] in {0: process, 1: update}, n[i] = samples consumed from `data`,
  out_len[i] (process only); expected = concatenated process outputs."""
import numpy as np

PROCESS, UPDATE = 0, 1


def flatten(ops):
    kind, n, out_len, data = [], [], [], []
    for op in ops:
        if op[0] == "process":
            x = np.asarray(op[1], np.float32)
            kind.append(PROCESS); n.append(x.size); out_len.append(op[2] if len(op) > 2 else x.size); data.append(x)
        else:
            r = np.asarray(op[1], np.float32)
            kind.append(UPDATE); n.append(r.size); out_len.append(0); data.append(r)
    return (np.array(kind, np.int32), np.array(n, np.int64), np.array(out_len, np.int64),
            np.concatenate(data) if data else np.zeros(0, np.float32))


def replay(conv, kind, n, out_len, data):
    outs, p = [], 0
    for k, m, o in zip(kind, n, out_len):
        chunk = data[p:p + m]
        p += m
        if k == PROCESS:
            outs.append(np.asarray(conv.process(chunk, int(o)) if o != m else conv.process(chunk), np.float32))
        else:
            conv.update(chunk)
    return np.concatenate(outs) if outs else np.zeros(0, np.float32)
