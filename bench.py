#!/usr/bin/env python3
"""Benchmark of the MI355X MapCrdt merge hot path (BASELINE.json metric).

Metric: merged records/sec (whole job, all ranks) on the 1024-replica fan-in
workload — 1B records, Zipf(0.8) keys over 2^28 ids, a 2^27-key local map —
plus the HBM-roofline fraction of the dominant kernel (K2 apply) and of the
whole job.  One "step" = one crdt_merge of the whole batch (R = 1024 sequential
Crdt.merge calls, crdt.dart:77-94) with every input already resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

N > 1, --scaling weak (default): the job is N x the single-GPU workload —
N·1B records, keys over N·2^28 ids sharded key % N, N·2^27 local keys; every
rank generates its own part (its 2^28 slots), changeset j is the rank-major
concatenation of the ranks' parts of replica j.  Per changeset one all-gather
of the part maxima (N x R int64) plus the MIN/MAX event reductions of
crdt_amd/dist.py::sharded_merge_parts — no records cross xGMI.
--scaling strong: the total stays 1B, keys sharded key % N, changeset j homed on
rank j % N (dist.py::sharded_merge, three int64 all-reduces).
Collectives are torch.distributed "nccl" = RCCL over xGMI.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12          # MI355X HBM3E, bytes/s (MI355X_MICROARCH.md chip table)
TIMING_EVERY = 8           # streaming configs (one merge call per delta): HIP-event timing sampled


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", choices=["fanin", "cfg2", "cfg3", "cfg5"], default="fanin")
    p.add_argument("--records", type=int, default=1_000_000_000)
    p.add_argument("--replicas", type=int, default=1024)
    p.add_argument("--keys", type=int, default=1 << 28)
    p.add_argument("--local", type=int, default=1 << 27)
    p.add_argument("--zipf", type=float, default=0.8)
    p.add_argument("--order", choices=["shuffled", "ascending"], default="shuffled")
    p.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    p.add_argument("--route", action="store_true",
                   help="N > 1: changeset j arrives whole on rank j %% N; records are routed to their owner "
                        "with RCCL all-to-all inside the timed step (north star config 4)")
    p.add_argument("--path", choices=["auto", "gather", "sorted"], default="auto",
                   help="merge strategy (crdt_set_merge_path): gather = K2 per changeset, sorted = key-partitioned")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU baseline sample")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-census", action="store_true", help="skip the distinct-key census (B_alg job)")
    p.add_argument("--no-pcie", action="store_true", help="skip the host-buffer (PCIe-inclusive) sample")
    p.add_argument("--exact-counts", action="store_true",
                   help="per-record n_present / n_won also on the sorted path (its changeset-ordered form)")
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_rank %= max(torch.cuda.device_count(), 1)          # gloo rehearsal: several ranks per GPU
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        # CRDT_BENCH_BACKEND=gloo: rehearsal of N ranks on one GPU (RCCL needs one GPU per rank)
        backend = os.environ.get("CRDT_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    from crdt_amd.dist import (sharded_merge, sharded_merge_parts, sharded_merge_routed, torch_all_gather,
                               torch_all_to_all, torch_alloc, torch_reducers)
    if world > 1:
        red_max, red_min = torch_reducers(dist)
        gather = torch_all_gather(dist)
        a2a = torch_all_to_all(dist)
        alloc = torch_alloc(dev)
    from crdt_amd import DeviceTable
    from crdt_amd.workload import gen_cfg2, gen_cfg3, gen_cfg5, gen_fanin

    t0 = time.time()
    weak = world > 1 and args.scaling == "weak"
    route = world > 1 and args.route
    if args.config == "fanin" and route:
        m = world if weak else 1
        wl = gen_fanin(total=args.records * m, R=args.replicas, K=args.keys * m, n_local=args.local * m,
                       s=args.zipf, device=dev, order=args.order, rank=rank, world=world, route=True)
        workload = (f"fanin routed x{world} ({'weak' if weak else 'strong'}): {wl['total']:,} records = "
                    f"{wl['R']} replicas x {wl['n_per_replica']:,}, replica j on rank j % {world}, Zipf({args.zipf}) "
                    f"keys over {m}·2^{int(np.log2(args.keys))} ids routed to owner key % {world} by RCCL "
                    f"all-to-all, local map {m}·2^{int(np.log2(args.local))} keys")
    elif args.config == "fanin" and weak:
        # this rank's part: a full single-GPU fan-in over its own 2^28 slots (global key = slot*N + rank)
        wl = gen_fanin(total=args.records, R=args.replicas, K=args.keys, n_local=args.local, s=args.zipf,
                       device=dev, order=args.order, rank=0, world=1, seed=0xC0FFEE04 + 7919 * rank)
        c0 = torch.tensor([wl["c0"]], dtype=torch.int64, device=dev)
        red_max(c0)                                               # refreshCanonicalTime of the whole map
        wl["c0"] = int(c0.item())
        cnt = torch.from_numpy(np.diff(wl["owned_offsets"].astype(np.int64))).to(dev)
        allc = gather(cnt).cpu().numpy()
        wl["index_base"] = allc[:rank].sum(axis=0) if rank else np.zeros(allc.shape[1], np.int64)
        wl["total"] = int(allc.sum())
        workload = (f"fanin weak x{world}: {wl['total']:,} records = {wl['R']} replicas x "
                    f"{world * wl['n_per_replica']:,}, per rank Zipf({args.zipf}) keys over its 2^"
                    f"{int(np.log2(args.keys))} slots of {world}·2^{int(np.log2(args.keys))} ids (key % N), "
                    f"{args.order} order, local map {world}·2^{int(np.log2(args.local))} keys")
    elif args.config == "fanin":
        wl = gen_fanin(total=args.records, R=args.replicas, K=args.keys, n_local=args.local, s=args.zipf,
                       device=dev, order=args.order, rank=rank, world=world)
        workload = (f"fanin: {wl['total']:,} records = {wl['R']} replicas x {wl['n_per_replica']:,}, "
                    f"Zipf({args.zipf}) keys over 2^{int(np.log2(args.keys))} ids (unique per replica, "
                    f"{args.order} order), local map 2^{int(np.log2(args.local))} keys, keys sharded key%N")
    elif args.config == "cfg2":
        assert world == 1, "cfg2 is a single-GPU configuration"
        wl = gen_cfg2(device=dev)
        workload = "cfg2: 10M-key local map + one 10M-record changeset, ~50% key overlap"
    elif args.config == "cfg3":
        assert world == 1, "cfg3 is a single-GPU configuration"
        wl = gen_cfg3(device=dev)
        workload = ("cfg3: 100M-key local map, 1024 replicas x 97,657 records, Zipf(1.0) keys, millis over 8 "
                    "values x counters over 4 (ties decided by node rank)")
    else:
        assert world == 1, "cfg5 runs on one GPU here"
        wl = gen_cfg5(device=dev)
        workload = ("cfg5 streaming: 100M-key table, 100 deltas x 10M records, one merge call per delta "
                    "(advancing wall), 10% tombstones, peers 1..16")
    torch.cuda.synchronize()
    log(f"workload generated in {time.time() - t0:.1f}s: {workload}")

    table = DeviceTable(local_rank, local_rank=0, capacity=wl["capacity"])
    table.set_merge_path(args.path)
    # per-record n_present / n_won are library extras (not reference results); without them the
    # sorted path folds each bucket in any order (same rows / canonical / status)
    table.set_counts(args.exact_counts)
    loc = wl["local"]
    own, home = wl["owned"], wl["home"]
    own_cols = (own["key"], own["lt"], own["rank"], own["val"], wl["owned_offsets"], None)
    if route:
        home_cols = (home["key"], home["lt"], home["rank"], home["val"], wl["home_offsets"], None)
    else:
        home_cols = (own["key"][:0] if world > 1 else own["key"], home["lt"], home["rank"],
                     own["val"][:0] if world > 1 else own["val"], wl["home_offsets"], None)
    R = wl["R"]
    d_max = torch.zeros(max(R, 1), dtype=torch.int64, device=dev)
    d_ev = torch.zeros(4, dtype=torch.int64, device=dev)

    def reset():
        table.clear_rows(0, wl["capacity"])
        table.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
        table.canonical = wl["c0"]
        torch.cuda.synchronize()

    def step(flags=None):
        if wl.get("per_call"):                       # streaming: one crdt_merge per delta
            offs, tot = wl["owned_offsets"], None
            for d in range(wl["R"]):
                b, e = int(offs[d]), int(offs[d + 1])
                fl = False if flags is None else flags[b:e]
                sample = table_timing[0] and d % TIMING_EVERY == 0      # HIP events on every 8th call only
                if table_timing[0]:
                    table.set_timing(sample)
                r, _ = table.merge(*delta_cols[d], int(wl["walls"][d]), win_flags=fl)
                if sample:
                    table_timing[1].append(table.timing())
                if tot is None:
                    tot = dict(r)
                else:
                    tot.update({k: r[k] for k in ("status", "canonical_lt", "exc_index", "drift_ms", "counter")})
                    tot["n_present"] += r["n_present"]
                    tot["n_won"] += r["n_won"]
                if r["status"] != 0:
                    break
            return tot
        if world == 1:
            res, _ = table.merge(*own_cols[:5], wl["wall"], win_flags=flags if flags is not None else False)
            return res
        if route:
            return sharded_merge_routed(table, home_cols, wl["wall"], d_max, d_ev, red_max, red_min, gather,
                                        a2a, rank, world, alloc, win_flags=flags)
        if weak:
            # per changeset: part scan -> all-gather maxima -> clock -> MIN(event) -> resolve -> MAX -> apply
            return sharded_merge_parts(table, own_cols, wl["wall"], wl["index_base"], d_max, d_ev, gather,
                                       red_max, red_min, rank, win_flags=flags)
        # key-sharded: home scan -> MAX(M_j) -> clock -> MIN(event) -> resolve -> MAX(details) -> apply
        return sharded_merge(table, home_cols, own_cols, wl["wall"], d_max, d_ev, red_max, red_min,
                             win_flags=flags)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # streaming deltas: the per-call column views and offsets are made once, outside the timed steps
    delta_cols = []
    if wl.get("per_call"):
        offs = wl["owned_offsets"]
        for d in range(wl["R"]):
            b, e = int(offs[d]), int(offs[d + 1])
            delta_cols.append((own["key"][b:e], own["lt"][b:e], own["rank"][b:e], own["val"][b:e],
                               np.array([0, e - b], np.uint64)))
    table_timing = [False, []]                     # per-call timing records (streaming config)
    for _ in range(args.warmup):
        reset()
        step()
    table.set_timing(True)
    table_timing[0] = True
    step_ms, apply_ms, apply_launches, apply_total, scan_ms, clock_ms, dev_ms = [], 0.0, 0, 0, 0.0, 0.0, 0.0
    res = None
    for _ in range(args.steps):
        reset()
        barrier()
        ts = time.perf_counter()
        res = step()
        barrier()
        dt = time.perf_counter() - ts
        if world > 1:
            t = torch.tensor([int(dt * 1e9)], device=dev, dtype=torch.int64)
            red_max(t)                                            # max over ranks (ns)
            dt = float(t.item()) / 1e9
        step_ms.append(dt * 1e3)
        tms, table_timing[1] = table_timing[1] or [table.timing()], []
        tm = {k: sum(t[k] for t in tms) for k in tms[0]}
        if wl.get("per_call"):                   # sampled calls -> per-step estimates
            f = wl["R"] / len(tms)
            for k in ("scan_ms", "clock_ms", "total_ms"):
                tm[k] *= f
            tm["apply_total"] = int(round(tm["apply_total"] * f))
        apply_ms += tm["apply_ms"]
        apply_launches += tm["apply_launches"]
        apply_total += tm["apply_total"]
        scan_ms += tm["scan_ms"]
        clock_ms += tm["clock_ms"]
        dev_ms += tm["total_ms"]
    table.set_timing(False)
    table_timing[0] = False
    assert res["status"] == 0, res
    ms_per_step = float(np.mean(step_ms))
    total_records = wl["total"]
    value = total_records / (ms_per_step / 1e3)

    # ---- per-kernel roofline of K2 (apply): algorithmic bytes / event-timed duration
    n_owned = int(res.get("n_recv", wl["owned_offsets"][-1]))            # routed: records received
    counts_known = res["n_present"] != (1 << 64) - 1                       # order-free sorted path: not counted
    kb = 20 * n_owned + (12 * res["n_present"] + 24 * res["n_won"] if counts_known else 0)   # per step, this rank
    launches_per_step = max(apply_total // max(args.steps, 1), 1)
    alg_per_launch = kb / launches_per_step
    avg_launch_us = apply_ms * 1e3 / max(apply_launches, 1)                  # HIP events, sampled launches
    achieved = alg_per_launch / (avg_launch_us / 1e6) if apply_ms > 0 else 0.0
    path = table.last_path()
    roofline = {"bound": "hbm", "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK, 4), "traffic": None,
                "kernel": "k_apply (K2)" if path == "gather" else
                "sorted apply: k_part_* x2 + k_resolve (one timed region per merge call)",
                "avg_launch_us": round(avg_launch_us, 2),
                "alg_bytes_per_launch": int(alg_per_launch), "launches_per_step": launches_per_step,
                "launches_timed": apply_launches}
    if path == "gather" and args.config == "fanin" and world == 1 and apply_ms > 0:
        # K2 against the measured ceiling of its own access pattern: random 16-B row reads
        # with 25 % of rows written back on a 2^28-row table (tools/ubench_rowwrite.hip)
        rate = (n_owned / launches_per_step) / (avg_launch_us / 1e6)
        roofline["pattern_ceiling"] = {"value": 30.4e9, "unit": "records/s", "achieved": round(rate, 1),
                                       "frac": round(rate / 30.4e9, 3),
                                       "source": "profiles/r01_ubench_rowwrite.txt"}
    # traffic (PMC) is filled from the committed rocprofv3 --pmc pass of this command, when present
    pmc = os.path.join(ROOT, "profiles", "pmc_k_apply.json")
    if os.path.exists(pmc) and world == 1 and args.config == "fanin":
        try:
            roofline["traffic"] = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:  # noqa: BLE001
            pass

    # ---- whole-job algorithmic bytes: distinct keys touched / won (one untimed census run)
    job = {}
    if not args.no_census and world == 1:
        reset()
        flags = torch.zeros(max(n_owned, 1), dtype=torch.uint8, device=dev)
        r2 = step(flags=flags) if world == 1 else None
        if wl.get("per_call"):      # every call is its own merge: U counted per call (= its records)
            u_touch, u_win = int(r2["n_present"]), int(r2["n_won"])
        else:
            keys = own["key"]
            all_keys = torch.unique(keys)
            u_touch = int((all_keys < wl["n_local_rows"]).sum().item()) if args.config in ("fanin", "cfg3") \
                else int((all_keys < wl["n_local"]).sum().item())
            del all_keys
            u_win = int(torch.unique(keys[flags[:n_owned].bool()]).numel())
        b_alg = 20 * total_records + 12 * u_touch + 24 * u_win
        job = {"U_touch": u_touch, "U_win": u_win, "B_alg_bytes": b_alg,
               "hbm_frac_job": round(b_alg / (ms_per_step / 1e3) / HBM_PEAK, 4),
               "records_won_total": int(r2["n_won"])}
        del flags
        if not counts_known and apply_ms > 0:
            # the sorted apply's bytes from the distinct-key counts (SURVEY 8(d)'s own terms)
            alg_per_launch = b_alg / launches_per_step
            achieved = alg_per_launch / (avg_launch_us / 1e6)
            roofline.update({"achieved": round(achieved / 1e9, 1), "frac": round(achieved / HBM_PEAK, 4),
                             "alg_bytes_per_launch": int(alg_per_launch),
                             "alg_bytes": "20 B x records + 12 B x U_touch + 24 B x U_win (distinct keys)"})

    # ---- CPU baseline (rank 0, N = 1): the C restatement of the reference algorithm
    cpu = cpu_omp = parity = None
    if rank == 0 and world == 1 and not args.no_cpu:
        if job:                        # the census merged with win flags: redo the timed path's merge
            reset()
            step()
            torch.cuda.synchronize()
        cpu = cpu_baseline(wl, args.cpu_seconds)
        cpu_omp, parity = cpu_baseline_omp(wl, args.cpu_seconds, table)
    pcie = None
    if rank == 0 and world == 1 and not args.no_pcie and not wl.get("per_call"):
        pcie = host_input_rate(table, wl, reset)

    out = {
        "metric": "merged records/sec (node) + % HBM roofline, 1B records x 1024 replicas",
        "value": round(value, 1), "unit": "records/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "weak" if (world == 1 or weak) else "strong", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
        "config": {"workload": workload, "records": total_records, "replicas": R,
                   "parallelism": (f"keyshard{world}-{'routed' if route else 'parts' if weak else 'home'}"
                                   if world > 1 else "single"), "merge_path": path,
                   "step_ms_all": [round(x, 3) for x in step_ms]},
        "roofline": roofline, "job": job, "cpu_baseline": cpu, "cpu_baseline_omp": cpu_omp, "parity": parity,
        "pcie_inclusive": pcie,
        "breakdown_ms": {"scan": round(scan_ms / args.steps, 3), "clock_verify_resolve": round(clock_ms / args.steps, 3),
                         "apply_kernels_est": round(avg_launch_us * launches_per_step / 1e3, 3),
                         "apply_launches": launches_per_step,
                         "device_total": round(dev_ms / args.steps, 3)},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    table.close()
    if parity is not None and not parity["equal"]:
        log(f"PARITY FAILURE against the CPU oracle: {parity}")
        sys.exit(3)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(wl, budget_s):
    """Times oracle/merge_oracle.c (faithful port: map copy per merge + clock read per record,
    single thread) on the first changesets of the same workload, within ~budget_s seconds."""
    import torch
    from oracle.oracle_c import OracleTable
    loc = wl["local"]
    cap = wl["capacity"]
    t = OracleTable(cap, 0, wl["c0"])
    t.put_rows(loc["slot"].cpu().numpy().astype(np.uint32), loc["lt"].cpu().numpy(),
               loc["rank"].cpu().numpy().astype(np.uint32), loc["val"].cpu().numpy().astype(np.uint32),
               loc["mod"].cpu().numpy())
    offs = wl["owned_offsets"]
    own = wl["owned"]
    done, recs, el = 0, 0, 0.0
    rows_copied = 0
    while done < wl["R"] and el < budget_s:
        b, e = int(offs[done]), int(offs[done + 1])
        sl = slice(b, e)
        cols = [own[k][sl].cpu().numpy() for k in ("key", "lt", "rank", "val")]
        ts = time.perf_counter()
        res, _ = t.merge(cols[0].astype(np.uint32), cols[1], cols[2].astype(np.uint32),
                         cols[3].astype(np.uint32), np.array([0, e - b], np.uint64),
                         int(wl["walls"][done]) if wl.get("per_call") else wl["wall"], faithful=True,
                         want_flags=False)
        el += time.perf_counter() - ts
        done += 1
        recs += e - b
        rows_copied += cap
    del t
    torch.cuda.synchronize()
    return {"value": round(recs / el, 1), "unit": "records/s", "cores": 1, "kind": "port",
            "sample": f"first {done} of {wl['R']} changesets ({recs:,} records) merged into the full "
                      f"{cap:,}-row map by oracle/merge_oracle.c in faithful mode (one full map copy per "
                      f"merge, map_crdt.dart:43; one clock read per record, hlc.dart:82), {el:.1f}s"}


def cpu_baseline_omp(wl, budget_s, table=None):
    """Times oracle/merge_omp.c (the optimised multi-core merge, same results) on the leading
    changesets of the same workload, 16 changesets per call, within ~budget_s seconds.

    When the sample covers the whole batch, the oracle's final state is also the full-size parity
    check of the GPU ``table`` (left by the timed path's last merge): every one of its rows and the
    canonical clock, bit for bit.  Returns (baseline, parity or None)."""
    import torch
    from oracle.oracle_c import OracleTable
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(os.cpu_count() or 1, 16)
    loc = wl["local"]
    t = OracleTable(wl["capacity"], 0, wl["c0"])
    t.put_rows(loc["slot"].cpu().numpy().astype(np.uint32), loc["lt"].cpu().numpy(),
               loc["rank"].cpu().numpy().astype(np.uint32), loc["val"].cpu().numpy().astype(np.uint32),
               loc["mod"].cpu().numpy())
    offs, own = wl["owned_offsets"], wl["owned"]
    per_call = wl.get("per_call", False)
    step = 1 if per_call else 16
    done, recs, el = 0, 0, 0.0
    while done < wl["R"] and el < budget_s:
        j1 = min(done + step, wl["R"])
        b, e = int(offs[done]), int(offs[j1])
        cols = [own[k][b:e].cpu().numpy() for k in ("key", "lt", "rank", "val")]
        sub = (offs[done:j1 + 1] - offs[done]).astype(np.uint64)
        wall = int(wl["walls"][done]) if per_call else wl["wall"]
        ts = time.perf_counter()
        res, _ = t.merge_omp(cols[0].astype(np.uint32), cols[1], cols[2].astype(np.uint32),
                             cols[3].astype(np.uint32), sub, wall, threads=threads, want_flags=False)
        el += time.perf_counter() - ts
        assert res.status == 0
        done = j1
        recs += e - b
    parity = None
    if table is not None and done == wl["R"]:
        parity = full_parity(table, t, wl["capacity"])
    del t
    torch.cuda.synchronize()
    return ({"value": round(recs / el, 1), "unit": "records/s", "cores": threads, "kind": "port",
             "sample": f"first {done} of {wl['R']} changesets ({recs:,} records) merged by oracle/merge_omp.c "
                       f"(parallel per-changeset max / apply, exact recv loop only on flagged changesets), "
                       f"{threads} OpenMP threads, {el:.1f}s"}, parity)


def host_input_rate(table, wl, reset, max_records: int = 128 << 20) -> dict:
    """The boundary as a dart:ffi caller uses it: columns in host memory, copied to the device
    inside crdt_merge.  Times one merge of the leading changesets (<= max_records records) from
    pageable numpy arrays and from pinned host tensors; reported beside `value`, never as it."""
    import torch
    offs, own = wl["owned_offsets"], wl["owned"]
    j1 = int(np.searchsorted(offs, max_records, side="right")) - 1
    j1 = max(1, min(j1, wl["R"]))
    n = int(offs[j1])
    sub = offs[:j1 + 1].astype(np.uint64)
    cols = [own[k][:n].cpu() for k in ("key", "lt", "rank", "val")]
    out = {"unit": "records/s", "records": n, "changesets": j1}
    for kind in ("pageable", "pinned"):
        hc = [c.clone() if kind == "pageable" else c.pin_memory() for c in cols]
        # numpy views of the same memory (int32 columns viewed as uint32, so nothing is re-copied)
        hc_np = [h.numpy().view(np.uint32) if h.dtype == torch.int32 else h.numpy() for h in hc]
        best = None
        for _ in range(2):
            reset()
            ts = time.perf_counter()
            res, _ = table.merge(*hc_np, sub, wl["wall"], win_flags=False)
            dt = time.perf_counter() - ts
            assert res["status"] == 0, res
            best = dt if best is None else min(best, dt)
        out[kind] = round(n / best, 1)
        out[kind + "_ms"] = round(best * 1e3, 2)
        del hc, hc_np
    out["sample"] = (f"first {j1} of {wl['R']} changesets ({n:,} records, {20 * n / 1e9:.2f} GB of columns) "
                     f"merged from host buffers: crdt_merge copies them to HBM, then runs the same path")
    return out


def full_parity(table, oracle, cap: int, chunk: int = 1 << 25) -> dict:
    """Every row of the GPU table (lt, rank, val, mod) and its canonical clock against the oracle's."""
    ts = time.perf_counter()
    bad = 0
    for b in range(0, cap, chunk):
        e = min(b + chunk, cap)
        got = table.read_rows(np.arange(b, e, dtype=np.uint32))
        ref = oracle.rows[b:e]
        for f, a in zip(("lt", "rank", "val", "mod"), got):
            bad += int(np.count_nonzero(a != ref[f]))
    canon = table.canonical == oracle.canonical
    return {"rows": cap, "fields_differing": bad, "canonical_equal": canon, "equal": bad == 0 and canon,
            "against": "oracle/merge_omp.c final state (tests pin it to oracle/merge_oracle.c)",
            "seconds": round(time.perf_counter() - ts, 1)}


if __name__ == "__main__":
    main()
