"""The host tier after batches, on the CPU (no GPU, no device calls): a tier holding a base copy plus
every later batch folded into its delta tree (csrc/host_tier.hpp, csrc/host_delta.hpp) answers rank,
select, rank-range and key-bound aggregates, key dumps and whole protocol rounds exactly as a tier
rebuilt from the merged contents.  The model folds batches with FingerprintTreeMap's semantics
(rsos/src/fingerprint_tree_map/mutate.rs:23-154): overwrite replaces, remove drops.

The driver (tests/host_tier_check.cpp) is compiled from the library's own headers with hipcc as a
host-only program."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "host_tier_check.cpp")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("htc") / "host_tier_check")
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    subprocess.run([hipcc, "-O2", "-std=c++17", "-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", SRC,
                    "-o", out], check=True)
    return out


CASES = [
    # kind (0 u32, 1 u64, 2 16-byte), seed, base rows, key universe, batches, largest batch
    (0, 1, 200, 300, 30, 40),
    (1, 2, 0, 500, 20, 100),         # empty base: every key an insertion
    (2, 3, 3000, 6000, 20, 900),     # byte keys sharing their leading 8 bytes
    (2, 7, 100000, 300000, 40, 8000),  # a tree of height 2, batches folded by single upserts
    (1, 8, 0, 400000, 30, 20000),      # large batches: merge-rebuilds
    (0, 9, 50000, 200000, 150, 300),   # many small batches into a large delta
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "k%d-s%d-b%d-u%d" % c[:4])
def test_tier_with_folded_batches_equals_rebuilt_tier(checker, case):
    r = subprocess.run([checker] + [str(x) for x in case], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["ok"] and res["checked"] > 0
