"""A/B a parity case against the oracle with the current library and another build
(CRDT_LIB_PATH), several repetitions each: tells a deterministic regression from a race.
  python tools/ab_case.py <other.so> [reps]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r'''
import sys, numpy as np
sys.path.insert(0, ROOT)
from crdt_amd import _capi
lib = __import__("ctypes").CDLL(_capi.LIB_PATH)
for n in list(_capi.SIGNATURES):
    if not hasattr(lib, n):
        del _capi.SIGNATURES[n]
from tests._cases import ABSENT_MOD, oracle_run
from tests.test_gpu_parity import _frame_edge_case
from crdt_amd import DeviceTable
bad = 0
for seed, slack, cap in [(91, 0, (1 << 20) + 3), (91, 0, None), (92, 1, (1 << 20) + 3)]:
    case = _frame_edge_case(seed)
    orows, ores, _ = oracle_run(case)
    for rep in range(REPS):
        t = DeviceTable(0, local_rank=case["local_rank"], capacity=cap or case["n_ids"])
        t.set_merge_path("sorted"); t.set_counts(False)
        if BOUND:
            t.set_rank_bound(int(case["rank"].max()) + 1 + slack)
        loc = case["local"]; keep = loc["mod"] != ABSENT_MOD
        ids = np.arange(case["n_local"], dtype=np.uint32)[keep]
        t.put_rows(ids, loc["lt"][keep], loc["rank"][keep], loc["val"][keep], loc["mod"][keep])
        t.canonical = case["c0"]
        t.merge(case["key"], case["lt"], case["rank"], case["val"], case["offsets"], case["wall"],
                millis=case["millis"], win_flags=False)
        rows = t.read_rows(np.arange(case["n_ids"], dtype=np.uint32))
        diff = [int((a != orows[f]).sum()) for f, a in zip(("lt", "rank", "val", "mod"), rows)]
        if any(diff):
            bad += 1
            x = np.nonzero(rows[0] != orows["lt"])[0][:3]
            print(f"  seed {seed} slack {slack} cap {cap} rep {rep}: diffs {diff} first rows {x.tolist()} "
                  f"dev {[int(rows[0][i]) for i in x]} ora {[int(orows['lt'][i]) for i in x]}")
        t.close()
print("mismatching runs:", bad)
'''

def main():
    other = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for lib in (None, other):
        for bound in (1, 0):
            env = dict(os.environ)
            if lib:
                env["CRDT_LIB_PATH"] = os.path.abspath(lib)
            code = CHILD.replace("ROOT", repr(ROOT)).replace("REPS", str(reps)).replace("BOUND", str(bound))
            print(f"== lib {lib or 'current'} rank_bound {'on' if bound else 'off'}", flush=True)
            r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, timeout=300)
            if r.returncode:
                sys.exit(r.returncode)

main()
