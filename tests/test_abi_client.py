"""The C ABI from a plain C program (reconcile-rs_amd/examples/abi_client.c): what the reference's
FFI binding would do -- host buffers in, host results out -- checked number by number against
the oracle (the FTM restatement and the literal rbsr driver) on the same records."""
import json
import os
import subprocess

import numpy as np
import pytest

import oracle as O
import rbsr as OR

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLIENT = os.path.join(ROOT, "reconcile-rs_amd", "examples", "abi_client")
M64 = (1 << 64) - 1


def splitmix64(state):
    while True:
        state = (state + 0x9E3779B97F4A7C15) & M64
        z = state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        yield z ^ (z >> 31)


def _recs(keys, vals):
    k = np.array(keys, np.uint64)
    v = np.array(vals, np.uint64)
    return O.Records(O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0), k.view(np.uint8).reshape(-1, 8),
                     v.view(np.uint8).reshape(-1, 8))


def _ftm(keys, vals):
    t = O.FingerprintTreeMap(_recs(keys, vals))
    t.fill(0, len(keys))
    return t


def _agg(d):
    return [int(x, 16) for x in d["fp"]], int(d["size"])


def test_client_is_built():
    assert os.access(CLIENT, os.X_OK), "make -C reconcile-rs_amd builds examples/abi_client"


@pytest.mark.gpu
def test_c_client_against_oracle(gpu, oracle_lib):
    n, seed = 200_000, 7
    out = subprocess.run([CLIENT, str(n), str(seed)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    got = json.loads(out.stdout)
    g = splitmix64(seed)
    keys = sorted(set(next(g) for _ in range(n)))
    m = len(keys)
    vals = [next(g) for _ in range(m)]
    t = _ftm(keys, vals)
    assert got["n"] == got["size"] == m
    assert _agg(got["root"]) == (list(t.root()[0]), m)
    probe = keys[m // 3] + 1
    assert got["probe"] == probe and got["rank_probe"] == t.rank(np.uint64(probe).tobytes())
    assert got["select_mid"] == keys[m // 2]
    fp, size = t.aggregate(np.uint64(keys[m // 4]).tobytes(), np.uint64(keys[3 * m // 4]).tobytes())
    assert _agg(got["range_q1_q3"]) == (list(fp), size)
    # the batch: inserts of the probe and two fresh keys, an overwrite, a delete
    bk = got["batch"]["keys"]
    assert bk[0] == probe and bk[3] == keys[10] and bk[4] == keys[20]
    content = dict(zip(keys, vals))
    new = sum(1 for k in bk[:3] if k not in content)
    for k, v in zip(bk[:4], [7, 8, 9, vals[10] + 1]):
        content[k] = v
    del content[keys[20]]
    assert (got["batch"]["new"], got["batch"]["overwritten"], got["batch"]["deleted"]) == (new, 1, 1)
    k2 = sorted(content)
    t2 = _ftm(k2, [content[k] for k in k2])
    assert _agg(got["root_after_batch"]) == (list(t2.root()[0]), len(k2))
    # the reconciliation: the literal driver over the two trees
    va, vb = OR.FtmView(t2, True), OR.FtmView(t, True)
    active, sides, rounds, segs, enum = OR.initial_ranges(va), [vb, va], 0, 0, 0
    while active:
        segs += len(active)
        ch, en = [], []
        OR.protocol_round(sides[rounds % 2], OR.fixed_fan_out(16), active, ch, en)
        enum += len(en)
        active, rounds = ch, rounds + 1
    assert got["reconcile"] == {"rounds": rounds, "segments": segs, "enumerated": enum}
