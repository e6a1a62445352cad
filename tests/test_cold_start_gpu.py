"""GPU: cold start (round-5 verdict item 4).

* cudasp_tf_prewarm (what the DuckDB extension runs in the background at
  LOAD) builds the fixed-base table and parks one ready streaming feed per
  GPU; the first query of the process then takes that feed, rebinds its keys
  and returns the reference SQL test's rows -- in a fresh process, so nothing
  was built before;
* a prewarm that finds its feed pooled adds nothing;
* the first query of a fresh process without prewarm is exact too (the
  feed and the table are built inside it)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_PROBE = r"""
import json, sys, time
sys.path[:0] = [%r, %r, %r]
import golden_io
from cudasp_amd import cudasp_scan, pool_size, prewarm
sc = golden_io.load("sql_cases.json")
q = sc["queries"][3]
table = [(bytes.fromhex(r["txid"]), r["height"], bytes.fromhex(r["tweak"]), r["outputs"])
         for r in sc["tables"]["test_data"] if r["height"] in (100, 200)]
out = {}
if sys.argv[1] == "prewarm":
    out["prewarm_s"] = prewarm()
    out["pool_after_prewarm"] = pool_size()
    out["prewarm_again_s"] = prewarm()
    out["pool_after_second_prewarm"] = pool_size()
t0 = time.perf_counter()
got = cudasp_scan(table, bytes.fromhex(q["scan_key"]), bytes.fromhex(q["spend_key"]),
                  [bytes.fromhex(l) for l in q["label_keys"]], stats=(st := {}))
out["first_query_s"] = time.perf_counter() - t0
out["heights"] = sorted(h for _, h, _ in got)
out["expected"] = q["expected"]
out["streaming_feeds"] = st.get("streaming_feeds")
out["pool_after_query"] = pool_size()
print(json.dumps(out))
"""


def _run(mode):
    code = _PROBE % (ROOT, os.path.join(ROOT, "duckdb-cudasp-extension_amd"), os.path.join(ROOT, "tests"))
    r = subprocess.run([sys.executable, "-c", code, mode], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_prewarmed_first_query_in_a_fresh_process():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = _run("prewarm")
    n = torch.cuda.device_count()
    assert d["pool_after_prewarm"] == n and d["pool_after_second_prewarm"] == n
    assert d["heights"] == d["expected"]
    assert d["streaming_feeds"] >= 1
    assert d["pool_after_query"] == n  # the query took the parked feed and gave it back


def test_first_query_without_prewarm_in_a_fresh_process():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = _run("cold")
    assert d["heights"] == d["expected"]
