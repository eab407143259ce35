cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for i in 1 2 3; do
  for v in early late; do
    a=""; [ $v = late ] && a="--late-alloc"
    timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu --no-pcie --no-census $a > gpurun_out/al_$v$i.json 2> gpurun_out/al_$v$i.log || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/al_$v$i.json')); print('$v$i', d['ms_per_step'], d['roofline']['dominant_kernel']['phases_ms_per_step'])"
  done
done
