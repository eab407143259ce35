#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/policy; mkdir -p $OUT
timeout -k 10 120 ./tools/ubench_policy > $OUT/times.txt 2>&1; rc=$?; cat $OUT/times.txt; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc -o run -- ./tools/ubench_policy > $OUT/pmc.log 2>&1; echo "pmc exit $?"
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/policy/pmc/*counter_collection.csv")[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if "k_policy" in r["Kernel_Name"]:
        aux = r["Kernel_Name"].split("<")[1].split(">")[0]
        acc[aux][r["Counter_Name"]].append(float(r["Counter_Value"]))
for aux, cs in sorted(acc.items(), key=lambda x: int(x[0])):
    print(aux, {c: round(sum(v)/len(v)/16.8e6, 3) for c, v in cs.items()}, "per row")
PY
