"""Repro attempt for DESIGN.md's round-3 claim that torch gathers and sorts of 10^8-row tensors
returned wrong rows on this image (commit 29d67a0).

Every op the round-3 debugging scripts (since removed) and bench.py's config5 path use on
10^8-row tensors is run on the GPU and checked against numpy on the host, on the same data:
  - torch.randperm(n, device="cuda", generator=...): a permutation of 0..n-1;
  - row gathers of a (n, 16) uint8 tensor by an int64 index (t[idx], index_select), and of its
    int64 view -- the shape of bench.py's overwrite rows (base["keys"][rows]) and of the test's
    expected-live-set assembly;
  - bool-mask nonzero() of n entries;
  - torch.sort / argsort(stable) of n int64 values (the lexsort keys of the expected set).
Prints one JSON line per check and a summary line; exit status 1 if any check disagrees.

  python scripts/torch_large_ops_repro.py [n]    (default n = 100_000_000)
"""
import json
import sys
import time

import numpy as np
import torch


def report(name, ok, **kw):
    print(json.dumps({"check": name, "ok": bool(ok), **kw}), flush=True)
    return bool(ok)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    dev = torch.device("cuda")
    results = []
    t0 = time.time()
    # keys: (n, 16) random bytes from a seeded host generator, uploaded once
    rng = np.random.default_rng(5)
    keys_np = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    keys = torch.from_numpy(keys_np).to(dev)
    torch.cuda.synchronize()

    # 1. randperm on the device (the round-3 scripts' row picks)
    g = torch.Generator(device=dev)
    g.manual_seed(9)
    perm = torch.randperm(n, generator=g, device=dev)
    perm_np = perm.cpu().numpy()
    cnt = np.bincount(perm_np, minlength=n)
    results.append(report("randperm_is_permutation", perm_np.min() == 0 and perm_np.max() == n - 1 and (cnt == 1).all(),
                          n=n, duplicates=int((cnt > 1).sum()), missing=int((cnt == 0).sum())))
    del cnt

    # 2. row gathers by an int64 index: a 1.8 M-row pick (bench / test shape) and a whole permutation
    for label, idx_np in (("pick_1m8", perm_np[:1_800_000]), ("full_perm", perm_np)):
        idx = torch.from_numpy(np.ascontiguousarray(idx_np)).to(dev)
        got = keys[idx].cpu().numpy()
        want = keys_np[idx_np]
        bad = np.nonzero((got != want).any(axis=1))[0]
        results.append(report("gather_rows_" + label, bad.size == 0, rows=int(idx_np.size), wrong_rows=int(bad.size),
                              first_wrong=int(bad[0]) if bad.size else None))
        got2 = torch.index_select(keys, 0, idx).cpu().numpy()
        bad2 = np.nonzero((got2 != want).any(axis=1))[0]
        results.append(report("index_select_" + label, bad2.size == 0, rows=int(idx_np.size), wrong_rows=int(bad2.size)))
        k64 = keys.view(torch.int64)  # (n, 2) int64 view, gathered the same way
        got3 = k64[idx].cpu().numpy()
        want3 = keys_np.view(np.int64)[idx_np]
        bad3 = np.nonzero((got3 != want3).any(axis=1))[0]
        results.append(report("gather_int64_view_" + label, bad3.size == 0, rows=int(idx_np.size),
                              wrong_rows=int(bad3.size)))
        del idx, got, got2, got3, want, want3
        torch.cuda.empty_cache()

    # 3. mask -> nonzero (the expected live set's kept rows)
    keep = torch.ones(n, dtype=torch.bool, device=dev)
    keep[torch.from_numpy(perm_np[:1_800_000]).to(dev)] = False
    kept = keep.nonzero().view(-1).cpu().numpy()
    keep_np = np.ones(n, bool)
    keep_np[perm_np[:1_800_000]] = False
    want_k = np.nonzero(keep_np)[0]
    results.append(report("mask_nonzero", kept.shape == want_k.shape and np.array_equal(kept, want_k),
                          rows=int(want_k.size), got_rows=int(kept.size)))
    del keep, kept, keep_np, want_k

    # 4. sort / stable argsort of n int64 (the big-endian leading words of the keys)
    hi_np = keys_np[:, :8].copy().view(">u8").ravel().astype(np.uint64).view(np.int64)
    hi = torch.from_numpy(hi_np).to(dev)
    sv, si = torch.sort(hi)
    sv_np = np.sort(hi_np)
    results.append(report("sort_values", np.array_equal(sv.cpu().numpy(), sv_np), n=n))
    si_np = si.cpu().numpy()
    results.append(report("sort_indices_consistent", np.array_equal(hi_np[si_np], sv_np), n=n))
    del sv, si, si_np
    torch.cuda.empty_cache()
    ai = torch.argsort(hi, stable=True).cpu().numpy()
    ai_np = np.argsort(hi_np, kind="stable")
    results.append(report("argsort_stable", np.array_equal(ai, ai_np), n=n))
    print(json.dumps({"summary": True, "n": n, "checks": len(results), "failed": results.count(False),
                      "torch": torch.__version__, "device": torch.cuda.get_device_name(0),
                      "seconds": round(time.time() - t0, 1)}), flush=True)
    return 0 if all(results) else 1


if __name__ == "__main__":
    sys.exit(main())
