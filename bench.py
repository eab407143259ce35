#!/usr/bin/env python3
"""Benchmark of the MI355X MapCrdt merge hot path (BASELINE.json metric).

Metric: merged records/sec (whole job, all ranks) on north-star config 4 — 1B records =
1024 replicas x 976,563, Zipf(0.8) keys over 2^28 ids, a 2^27-key local map — plus the
HBM-roofline fraction of the job (B_alg = 20 B x records + 12 B x U_touch
+ 24 B x U_win over distinct keys, / step time / (N x 8 TB/s)).  One "step" = one
crdt_merge of the whole batch (R = 1024 sequential Crdt.merge calls, crdt.dart:77-94)
with every input already resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

N = 1: one ctx merges the whole batch.
N > 1 (strong scaling, config 4): the SAME 1B records; replica j arrives whole on rank
j % N, keys are owned by rank key % N.  Every rank's ctx is joined to an RCCL
communicator (crdt_comm_init_rccl) and the step is one collective crdt_merge per rank:
the library all-gathers the part maxima, reduces the first exception, routes every
record to its owner in one grouped all-to-all over xGMI and applies what it owns
(crdt_amd/csrc/comm_path.inc).  value = 1,000,000,512 / max-over-ranks step time.  The
pre-sharded figure (every rank already holding exactly the records it owns: no record
exchange) is reported beside it under "presharded".
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
PMC_FILE = os.path.join(ROOT, "profiles", "r06_pmc_bench.json")    # rocprofv3 --pmc of the default command


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


class GpuSampler:
    """GPU clock / power / temperature sampled from the card's hwmon during the timed steps (no privileges
    needed): freq1 = the graphics clock, freq2 = the memory clock, power1 = board power, temp2 / temp3.
    Per step: mean / min / max of each, so a slow step or process can be matched with its clocks."""

    FILES = {"sclk_mhz": ("freq1_input", 1e-6), "mclk_mhz": ("freq2_input", 1e-6), "power_w": ("power1_input", 1e-6),
             "temp_edge_c": ("temp2_input", 1e-3), "temp_hot_c": ("temp3_input", 1e-3)}

    def __init__(self, dev_index: int):
        import glob
        import threading
        self.dir = None
        try:
            import torch
            pr = torch.cuda.get_device_properties(dev_index)
            slot = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
            hw = glob.glob(f"/sys/bus/pci/devices/{slot}/hwmon/hwmon*")
            self.dir, self.slot = (hw[0] if hw else None), slot
        except Exception:  # noqa: BLE001 -- no sampler on this box
            self.dir = None
        self.samples, self.marks = [], []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _read(self):
        out = {}
        for k, (f, sc) in self.FILES.items():
            try:
                with open(f"{self.dir}/{f}") as fh:
                    out[k] = int(fh.read()) * sc
            except (OSError, ValueError):
                pass
        return out

    def _run(self):
        while not self._stop.is_set():
            self.samples.append((time.perf_counter(), self._read()))
            time.sleep(0.002)

    def start(self):
        if self.dir:
            self._t.start()
        return self

    def mark(self, t0: float, t1: float):
        self.marks.append((t0, t1))

    def stop(self) -> dict | None:
        if not self.dir:
            return None
        self._stop.set()
        self._t.join(timeout=2)
        steps = []
        for t0, t1 in self.marks:
            win = [v for t, v in self.samples if t0 <= t <= t1]
            st = {"samples": len(win)}
            for k in self.FILES:
                xs = [v[k] for v in win if k in v]
                if xs:
                    st[k] = [round(float(np.mean(xs)), 1), round(float(np.min(xs)), 1), round(float(np.max(xs)), 1)]
            steps.append(st)
        return {"source": f"{self.dir} (PCI {self.slot})", "per_step": steps,
                "fields": "[mean, min, max] over the samples inside each timed step (~2 ms apart)"}


class Heartbeat:
    """A line on stderr (rank 0) every `every` seconds while a long phase runs — full-size N > 1 rehearsals
    (several ranks generating 1B records on one GPU, host-staged exchanges) go minutes between log lines."""

    def __init__(self, every: float = 45.0):
        import threading
        self.phase = "start"
        self.t0 = time.time()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, args=(every,), daemon=True)
        self._t.start()

    def _run(self, every):
        while not self._stop.wait(every):
            log(f"... {self.phase} ({time.time() - self.t0:.0f} s)")

    def stop(self):
        self._stop.set()


class Watchdog:
    """Every rank's bound on one collective merge call (N > 1).  The library ends a call
    whose peer is lost at its own deadline (crdt_set_comm_timeout: CRDT_E_COMM); this catches what it cannot
    see — a rank stuck outside a collective merge, or inside RCCL's host calls (connection setup).  When a
    call overruns it prints this rank's phase, the library's phase and last plan, and exits the process
    non-zero (os._exit: no exec), so the launcher ends the job with a diagnosis instead of a timeout."""

    def __init__(self, rank: int):
        import threading
        self.rank = rank
        self.table = None
        self.what = None
        self.deadline = None
        self._lock = threading.Lock()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def arm(self, seconds: float, what: str):
        with self._lock:
            self.what, self.deadline = what, time.monotonic() + seconds

    def disarm(self):
        with self._lock:
            self.deadline = None

    def _run(self):
        while True:
            time.sleep(0.5)
            with self._lock:
                late = self.deadline is not None and time.monotonic() > self.deadline
                what = self.what
            if not late:
                continue
            lib = plan = None
            try:
                lib = self.table.comm_state() if self.table is not None else None
                plan = self.table.last_plan() if self.table is not None else None
            except Exception as e:  # noqa: BLE001 -- the report must go out whatever the table's state
                lib = f"unreadable: {e!r}"
            print(f"[bench] rank {self.rank}: WATCHDOG: {what} overran its bound; library (state, phase) {lib}; "
                  f"last plan {plan}", file=sys.stderr, flush=True)
            os._exit(4)


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
    p.add_argument("--millis-span", type=int, default=1 << 16,
                   help="fan-in: replica clocks drawn over this many ms (2^26: replicas ~18 h apart)")
    p.add_argument("--path", choices=["auto", "gather", "sorted"], default="auto",
                   help="merge strategy (crdt_set_merge_path): gather = K2 per changeset, sorted = key-partitioned")
    p.add_argument("--no-presharded", action="store_true", help="N > 1: skip the pre-sharded figure")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of each CPU baseline sample")
    p.add_argument("--cpu-changesets", type=int, default=64, help="changesets of the faithful CPU port's sample")
    p.add_argument("--no-cpu-copy16", action="store_true",
                   help="skip cpu_baseline_copy16 (the faithful port with its map copy on 16 threads)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-census", action="store_true", help="skip the distinct-key census (B_alg job)")
    p.add_argument("--flag-steps", type=int, default=2,
                   help="steps of the same merge with per-record win flags, timed after the census (N = 1)")
    p.add_argument("--no-pcie", action="store_true", help="skip the host-buffer (PCIe-inclusive) sample")
    p.add_argument("--exact-counts", action="store_true",
                   help="per-record n_present / n_won also on the sorted path (its changeset-ordered form)")
    p.add_argument("--row-bytes", type=int, choices=[0, 24, 32], default=0,
                   help="device row size (crdt_set_row_bytes); 0: 32 for the gather-path streaming configs "
                        "(cfg2, cfg5: random winner writes), else 24")
    p.add_argument("--late-alloc", action="store_true",
                   help="create the table after the workload (the library allocates its scratch in the first merge)")
    p.add_argument("--comm-timeout", type=float, default=120.0,
                   help="N > 1: one collective merge's deadline in s inside the library (crdt_set_comm_timeout)")
    p.add_argument("--call-timeout", type=float, default=300.0,
                   help="N > 1: every rank's watchdog bound on one merge call in s (then it reports and exits)")
    p.add_argument("--dist-timeout", type=float, default=1800.0,
                   help="N > 1: torch.distributed's timeout in s (barriers, the parity gather)")
    p.add_argument("--ab", default=None, metavar="VAR=v1,v2",
                   help="development A/B: the timed steps alternate the library switch VAR over the values "
                        "(one process, one memory placement); per-value step times go to stderr")
    return p.parse_args()


def main():
    args = parse()
    ab = None
    if args.ab:
        var, vals = args.ab.split("=", 1)
        ab = (var, vals.split(","), {})
        os.environ["CRDT_ENV_DYNAMIC"] = "1"        # the library re-reads its switches per merge
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        os.environ["CRDT_ENV_DYNAMIC"] = "1"         # route_ab below switches the routing per merge
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_rank %= max(torch.cuda.device_count(), 1)          # gloo rehearsal: several ranks per GPU
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    # CRDT_BENCH_BACKEND=gloo: rehearsal of N ranks on one GPU (RCCL needs one GPU per rank); the
    # library then exchanges through dist.GlooComm (host-staged) instead of its RCCL communicator
    backend = os.environ.get("CRDT_BENCH_BACKEND", "nccl")
    watchdog = None
    if world > 1:
        import datetime
        to = datetime.timedelta(seconds=args.dist_timeout)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=to)
        else:
            dist.init_process_group(backend, timeout=to)
        watchdog = Watchdog(rank)
    from crdt_amd import DeviceTable
    from crdt_amd.dist import GlooComm, attach_rccl
    from crdt_amd.workload import gen_cfg2, gen_cfg3, gen_cfg5, gen_fanin

    beat = Heartbeat()
    beat.phase = "creating the table"

    def all_max(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def all_sum(x: int) -> int:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return int(t.item())

    # the fan-in's table and partition scratch are allocated before the workload, while device
    # memory is unfragmented (the library's big buffers then sit in few large fragments)
    table = None
    if args.config == "fanin" and not args.late_alloc:
        table = DeviceTable(local_rank, local_rank=0, capacity=-(-args.keys // world))
        table.reserve_scratch(args.records if world == 1 else int(args.records / world * 1.25))
        torch.cuda.synchronize()

    beat.phase = "generating the workload"
    t0 = time.time()
    census = args.config == "fanin" and not args.no_census and world > 1      # N > 1: counted at generation
    # gloo rehearsal (several ranks on ONE GPU): the ranks generate their workloads one after another —
    # heavy kernels of eight processes time-sliced on one GPU took over 18 minutes for the 1B fan-in
    serial_gen = world > 1 and backend != "nccl"
    for r_ in range(world if serial_gen else 1):
        if serial_gen:
            dist.barrier()
            log(f"generating rank {r_}'s workload ({time.time() - t0:.0f} s)")
            if r_ != rank:
                continue
        wl, workload = make_workload(args, dev, rank, world, census)
    if serial_gen:
        dist.barrier()
    torch.cuda.synchronize()
    log(f"workload generated in {time.time() - t0:.1f}s: {workload}")

    if table is None:
        table = DeviceTable(local_rank, local_rank=0, capacity=wl["capacity"])
    assert table.capacity >= wl["capacity"]
    row_bytes = args.row_bytes or (32 if args.config in ("cfg2", "cfg5") else 24)
    table.set_row_bytes(row_bytes)
    table.set_merge_path(args.path)
    # per-record n_present / n_won are library extras (not reference results); without them the
    # sorted path folds each bucket in any order (same rows / canonical / status)
    table.set_counts(args.exact_counts)
    # node ranks are dense host-interned ids (replica j is rank j + 1, local rows 0 .. R): the
    # sorted path takes its packed key's rank frame from this bound instead of a pass over ranks
    table.set_rank_bound(wl["R"] + 1 if args.config in ("fanin", "cfg3") else 0)
    if world > 1:
        if backend == "nccl":
            attach_rccl(table, dist)                 # RCCL communicator inside the ctx
        else:
            table.comm_init_ops(world, rank, GlooComm(dist))
        # a lost peer ends a call at this deadline (CRDT_E_COMM) on every surviving rank; the watchdog bounds
        # the whole call on each rank
        table.set_comm_timeout(int(args.comm_timeout * 1e3))
        watchdog.table = table
    loc = wl["local"]
    src = wl["home"] if world > 1 else wl["owned"]
    offs = wl["home_offsets"] if world > 1 else wl["owned_offsets"]
    cols = (src["key"], src["lt"], src["rank"], src["val"], offs)
    R = wl["R"]

    def reset():
        table.clear_rows(0, wl["capacity"])
        table.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
        table.canonical = wl["c0"]
        torch.cuda.synchronize()

    def step(flags=None):
        if watchdog is not None:
            watchdog.arm(args.call_timeout, f"merge step ({beat.phase})")
        try:
            return step_(flags)
        finally:
            if watchdog is not None:
                watchdog.disarm()

    def step_(flags=None):
        if wl.get("per_call"):                       # streaming: one crdt_merge per delta
            tot = None
            for d in range(wl["R"]):
                b, e = int(offs[d]), int(offs[d + 1])
                fl = False if flags is None else flags[b:e]
                sample = table_timing[0] and d % TIMING_EVERY == 0      # HIP events on every 8th call only
                if watchdog is not None:
                    watchdog.arm(args.call_timeout, f"merge of delta {d} ({beat.phase})")
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
        res, _ = table.merge(*cols, wl["wall"], win_flags=flags if flags is not None else False)
        return res

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # streaming deltas: the per-call column views and offsets are made once, outside the timed steps
    delta_cols = []
    if wl.get("per_call"):
        for d in range(wl["R"]):
            b, e = int(offs[d]), int(offs[d + 1])
            delta_cols.append((src["key"][b:e], src["lt"][b:e], src["rank"][b:e], src["val"][b:e],
                               np.array([0, e - b], np.uint64)))
    table_timing = [False, []]                     # per-call timing records (streaming config)
    ab_ph = {}                                     # A/B: per-value phase timings of each step
    step_phases = []                               # every timed step's phase timings

    def timed_run(steps, sampler=None):
        step_ms, tsum, res = [], {}, None
        table.set_timing(True)
        table_timing[0] = True
        for si in range(steps):
            if ab:
                os.environ[ab[0]] = ab[1][si % len(ab[1])]
            reset()
            barrier()
            ts = time.perf_counter()
            res = step()
            barrier()
            te = time.perf_counter()
            if sampler:
                sampler.mark(ts, te)
            step_ms.append(all_max(te - ts) * 1e3)       # max over ranks
            if world > 1:
                log(f"timed step {si}: {step_ms[-1]:.1f} ms")
            if ab:
                ab[2].setdefault(ab[1][si % len(ab[1])], []).append(step_ms[-1])
            tms, table_timing[1] = table_timing[1] or [table.timing()], []
            tm = {k: sum(t[k] for t in tms) for k in tms[0]}
            if wl.get("per_call"):                   # sampled calls -> per-step estimates
                f = wl["R"] / len(tms)
                for k in ("scan_ms", "clock_ms", "route_ms", "total_ms", "sent_bytes"):
                    tm[k] *= f
                tm["apply_total"] = int(round(tm["apply_total"] * f))
            for k, v in tm.items():
                tsum[k] = tsum.get(k, 0) + v
            step_phases.append(tm)
            if ab:
                ab_ph.setdefault(ab[1][si % len(ab[1])], []).append(tm)
        table.set_timing(False)
        table_timing[0] = False
        return step_ms, tsum, res

    # N > 1 fan-in: the library's routing tuner (comm_path.inc RouteTune) takes its trial calls — each way of
    # moving the records twice (route_l1 in 2 pieces, the combine, route_l1 in 4 and in 1, route_l1 with the head
    # fold), the fastest kept — before
    # the warmup, so every timed step takes the chosen way
    beat.phase = "merging"
    route_tune = None
    if world > 1 and args.config == "fanin" and os.environ.get("CRDT_ROUTE_TUNE", "1") != "0":
        for i in range(12):
            reset()
            ts = time.perf_counter()
            step()
            log(f"routing tuner call {i}: {(time.perf_counter() - ts) * 1e3:.1f} ms, plan {table.last_plan()}")
            if table.route_tune()["best"] is not None:
                break
        route_tune = table.route_tune()
        log(f"routing tuner: {route_tune}")
    # N = 1 fan-in: the library's placement tuner (crdt_reserve_scratch took candidate level-1 buffers) times
    # the level-1 scatter on each in the first merges and keeps the fastest — also before the warmup
    placement = None
    if world == 1 and table.place_info()["candidates"] > 1:
        for _ in range(10):                              # (a warm-up merge, then two per candidate)
            before = table.place_info()
            if before["kept"] is not None:
                break
            reset()
            step()
            if table.place_info()["merges_used"] == before["merges_used"]:
                break                                    # (this path does not partition: nothing to time)
        placement = table.place_info()
        log(f"placement tuner: {placement}")
    for i in range(args.warmup):
        reset()
        ts = time.perf_counter()
        step()
        if world > 1:
            log(f"warmup {i}: {(time.perf_counter() - ts) * 1e3:.1f} ms")
    sampler = GpuSampler(local_rank).start()
    step_ms, tsum, res = timed_run(args.steps, sampler)
    gpu_clocks = sampler.stop()
    if gpu_clocks is not None and world == 1:       # this process's streaming copy rate (a 4 GiB device copy)
        a = torch.empty(1 << 30, dtype=torch.int32, device=dev)
        b = torch.empty_like(a)
        b.copy_(a)
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for _ in range(5):
            b.copy_(a)
        torch.cuda.synchronize()
        gpu_clocks["copy_GBs"] = round(5 * 2 * a.numel() * 4 / (time.perf_counter() - ts) / 1e9, 1)
        del a, b
        torch.cuda.empty_cache()
    if gpu_clocks:                                  # each step's time and level-1 scatter beside its clocks
        for st, ms, ph in zip(gpu_clocks["per_step"], step_ms, step_phases):
            st["step_ms"] = round(ms, 3)
            st["part1_ms"] = round(ph.get("part1_ms", 0.0), 3)
    plan = table.last_plan()                        # (later merges — census, samples — may go elsewhere)
    if ab:
        for v, ms in ab[2].items():
            log(f"A/B {ab[0]}={v}: mean {np.mean(ms):.3f} ms  min {np.min(ms):.3f}  max {np.max(ms):.3f}  "
                f"({len(ms)} steps)")
            ph = ab_ph.get(v, [])
            if ph:
                log(f"A/B {ab[0]}={v} phases: " + "  ".join(
                    f"{k} {np.mean([t[k] for t in ph]):.3f}" for k in ph[0]
                    if k.endswith("_ms") and isinstance(ph[0][k], (int, float))))
        os.environ.pop(ab[0], None)
    assert res["status"] == 0, res
    ms_per_step = float(np.mean(step_ms))
    total_records = wl["total"]
    value = total_records / (ms_per_step / 1e3)
    path = table.last_path()
    K = args.steps

    # ---- whole-job algorithmic bytes: distinct keys touched / won
    job = {}
    with_flags = None
    if not args.no_census and wl.get("per_call"):
        # streaming: every call is its own merge, so U is counted per call (= its records)
        reset()
        r2 = step(flags=torch.zeros(max(total_records, 1), dtype=torch.uint8, device=dev))
        u_touch, u_win = int(r2["n_present"]), int(r2["n_won"])
        job["census"] = "per call: U_touch = records whose key was present, U_win = records stored"
    elif not args.no_census and world == 1:
        # U_touch: distinct batch keys present in the local map; U_win: distinct keys of the stored
        # records (win flags of one untimed census merge) — bitmaps over the key space, in chunks
        reset()
        flags = torch.zeros(max(total_records, 1), dtype=torch.uint8, device=dev)
        r2 = step(flags=flags)
        seen = torch.zeros(wl["capacity"], dtype=torch.bool, device=dev)
        won = torch.zeros(wl["capacity"], dtype=torch.bool, device=dev)
        for b in range(0, total_records, 1 << 27):
            k = src["key"][b:b + (1 << 27)].long()
            seen[k] = True
            won[k[flags[b:b + (1 << 27)].bool()]] = True
            del k
        present = torch.zeros(wl["capacity"], dtype=torch.bool, device=dev)
        present[loc["slot"].long()] = loc["mod"] >= 0
        u_touch, u_win = int((seen & present).sum().item()), int(won.sum().item())
        del seen, won, present
        job["records_won_total"] = int(r2["n_won"])
        job["census"] = ("U_touch = distinct batch keys present in the local map, U_win = distinct keys of the "
                         "records stored (win flags of one untimed merge)")
        # the same merge with per-record win flags (what Crdt.merge's removeWhere / watch need,
        # crdt.dart:80-90): timed like the headline steps, beside it
        if args.flag_steps > 0:
            fl_ms = []
            for _ in range(args.flag_steps):
                reset()
                barrier()
                ts = time.perf_counter()
                r3 = step(flags=flags)
                barrier()
                fl_ms.append((time.perf_counter() - ts) * 1e3)
            assert r3["status"] == 0 and r3["canonical_lt"] == res["canonical_lt"], (r3, res)
            fm = float(np.mean(fl_ms))
            fpath, fplan = table.last_path(), table.last_plan()
            with_flags = {"ms_per_step": round(fm, 3), "value": round(total_records / (fm / 1e3), 1),
                          "unit": "records/s", "merge_path": fpath, "flagged_form": bool(fplan.get("flagged")),
                          "step_ms_all": [round(x, 3) for x in fl_ms],
                          "what": "same job with a 1-B win flag per record (crdt_merge win_flags, what Crdt.merge's "
                                  "removeWhere and watch() need): the sorted path's flagged form (stable level 2, "
                                  "ordered resolve, flags carried back to input order; DESIGN 5.4)"}
            if fpath == "sorted" and not args.no_cpu:
                # the same merge on the gather path (K2 decides each record in changeset order): its
                # flags, counts and canonical must equal the flagged form's, record for record
                reset()
                g_flags = torch.zeros_like(flags)
                table.set_merge_path("gather")
                ts = time.perf_counter()
                r4 = step(flags=g_flags)
                torch.cuda.synchronize()
                g_ms = (time.perf_counter() - ts) * 1e3
                table.set_merge_path(args.path)
                with_flags["gather_ms"] = round(g_ms, 3)
                with_flags["flags_equal_gather"] = bool(torch.equal(g_flags, flags))
                with_flags["counts_equal_gather"] = (r4["n_won"], r4["n_present"]) == (r3["n_won"], r3["n_present"])
                del g_flags
        del flags
    elif census:
        u_touch = all_sum(wl["u_touch"])
        # U_win: rows the merge stamped — mod >= c0 after the timed merge, less the local rows
        # whose lt (= mod) is c0 (the only local rows that can carry it): exact up to those few
        since = table.modified_since(wl["capacity"], wl["c0"])
        local_at_c0 = int((loc["mod"] == wl["c0"]).sum().item())
        u_win = all_sum(len(since) - local_at_c0)
        job["census"] = ("U_touch = distinct batch keys present in the local map (bitmap at generation), "
                         "U_win = rows stamped by the merge (mod >= C_0, crdt_modified_since) less the local "
                         "rows at C_0; both summed over ranks")
    if "census" in job:
        b_alg = 20 * total_records + 12 * u_touch + 24 * u_win
        job.update({"U_touch": u_touch, "U_win": u_win, "B_alg_bytes": b_alg,
                    "hbm_frac_job": round(b_alg / (ms_per_step / 1e3) / (world * HBM_PEAK), 4)})

    # ---- roofline: the contract fraction of the whole step (B_alg / t / (N x 8 TB/s)); the
    # dominant kernel's own per-launch figure beside it
    apply_ms = tsum.get("apply_ms", 0.0)
    apply_launches = max(int(tsum.get("apply_launches", 0)), 1)
    launches_per_step = max(int(tsum.get("apply_total", 0)) // max(K, 1), 1)
    avg_launch_us = apply_ms * 1e3 / apply_launches
    roofline = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": None,
                "traffic": None,
                "scope": "whole step: B_alg (SURVEY 8(d), distinct keys) / step time / N GPUs"}
    if job:
        ach = job["B_alg_bytes"] / (ms_per_step / 1e3) / world
        roofline.update(achieved=round(ach / 1e9, 1), frac=round(ach / HBM_PEAK, 4))
    if path == "gather" and apply_ms > 0 and res["n_present"] != (1 << 64) - 1:
        # K2 per launch on its own records (20 B each + 12 B per present + 24 B per won record,
        # counted per record, i.e. repeated writes of a key in several changesets included)
        n_mine = int(offs[-1]) if world == 1 else None
        if n_mine is not None:
            kb = (20 * n_mine + 12 * res["n_present"] + 24 * res["n_won"]) / launches_per_step
            roofline["dominant_kernel"] = {
                "kernel": "k_apply (K2)", "avg_launch_us": round(avg_launch_us, 2), "launches_per_step":
                launches_per_step, "alg_bytes_per_launch": int(kb),
                "achieved_GBs": round(kb / (avg_launch_us / 1e6) / 1e9, 1),
                "frac": round(kb / (avg_launch_us / 1e6) / HBM_PEAK, 4),
                "note": "per-record bytes (a key written by several changesets counts each time)"}
        if args.config == "fanin" and world == 1:
            rate = (int(offs[-1]) / launches_per_step) / (avg_launch_us / 1e6)
            roofline["self_ubench_ceiling"] = {
                "what": "K2's rate against the builder's own microbenchmark of its access pattern "
                        "(random 16-B row reads, 25 % written back, 2^28 rows) -- not a roofline",
                "value": 30.4e9, "unit": "records/s", "achieved": round(rate, 1), "frac": round(rate / 30.4e9, 3),
                "source": "profiles/r01_ubench_rowwrite.txt"}
    elif path == "sorted" and apply_ms > 0:
        # the level-1 partition scatter (one launch per step, HIP events around it).  Contract bytes
        # (SURVEY 8(d)): the 20 B of every record it reads; its partition record (packed 12 B + key
        # column, or 16 + 4 B) is scratch, reported separately with the PMC traffic of the kernel
        out_b = (12 + 2) if plan["key16"] else (12 + 4) if plan["packed"] else (16 + 4)
        p1_us = tsum.get("part1_ms", 0.0) * 1e3 / K
        n_app = int(tsum.get("part1_records", 0)) // max(K, 1)
        dk = {"kernel": "k_part_scatter1 (level-1 partition, one launch per step)",
              "phases_ms_per_step": {k: round(tsum.get(f"{k}_ms", 0.0) / K, 3)
                                     for k in ("scan", "part1", "part2", "resolve")},
              "apply_ms_per_step": round(apply_ms / K, 3), "plan": plan}
        if p1_us > 0 and n_app:
            kb = n_app * 20
            dk.update({"avg_launch_us": round(p1_us, 1), "alg_bytes_per_launch": kb,
                       "records_per_launch": n_app,
                       "bytes_per_record": f"20 read (SURVEY 8(d)); + {out_b} B scratch written, not counted",
                       "achieved_GBs": round(kb / (p1_us / 1e6) / 1e9, 1),
                       "frac": round(kb / (p1_us / 1e6) / HBM_PEAK, 4)})
            pk = pmc_kernel(args, path, "k_part_scatter1", world)
            if pk:
                tb = pk["read_bytes_per_step"] + pk["write_bytes_per_step"]
                dk.update({"actual_traffic_bytes": int(tb), "actual_traffic_source": pk["source"],
                           "actual_traffic_frac": round(tb / (p1_us / 1e6) / HBM_PEAK, 4)})
        roofline["dominant_kernel"] = dk
    # traffic: HBM bytes per step from this round's rocprofv3 --pmc passes of this exact command
    pm = pmc_profile(args, path, world)
    if pm:
        roofline["traffic"] = pm["hbm_bytes_per_step"]
        roofline["traffic_source"] = os.path.relpath(PMC_FILE, ROOT)

    beat.phase = "baselines and parity"
    cpu = cpu16 = cpu_omp = parity = None
    if world > 1 and args.config in ("fanin", "cfg5") and not args.no_cpu:
        # N > 1: every rank digests its shard (one 64-bit word per 2^20 slots, after the timed path's
        # last merge); rank 0 regenerates the same batch unsharded, times the CPU baselines on it and
        # runs the OpenMP oracle over all of it, then compares every shard's digests and the
        # canonical with the oracle's state (the other ranks wait at the barrier)
        dig = shard_digests(table, wl["capacity"])
        mine = (rank, dig.tolist(), int(table.canonical))
        got = [None] * world
        dist.all_gather_object(got, mine)
        if rank == 0:
            if args.config == "fanin":
                full = gen_fanin(total=args.records, R=args.replicas, K=args.keys, n_local=args.local, s=args.zipf,
                                 device=dev, order=args.order, millis_span=args.millis_span)
            else:
                full = gen_cfg5(device=dev)
            cpu = cpu_baseline(full, args.cpu_seconds, args.cpu_changesets, threads=1)
            if not args.no_cpu_copy16:
                cpu16 = cpu_baseline(full, args.cpu_seconds, args.cpu_changesets)
            cpu_omp, _, oracle = cpu_baseline_omp(full, args.cpu_seconds, keep=True)
            del full
            torch.cuda.empty_cache()
            parity = shard_parity(oracle, got, world) if oracle is not None else None
            del oracle
        barrier()
    # ---- N > 1: one timed step in each way of moving the records (the same job; CRDT_ENV_DYNAMIC):
    # route_l1 = home records partitioned straight into the owners' level-1 buckets (14-B level-1
    # records over the exchange, owners from level 2 on), combine = the map-side fold first (16-B
    # packed maxima), route = plain record routing (owners run the whole sorted path), route_l1_head = route_l1
    # with every owner's first level-1 digit folded at the sender; DESIGN §7
    route_ab = None
    if world > 1 and args.config == "fanin":
        route_ab = {"default_plan": {k: v for k, v in plan.items()
                                     if k in ("route_l1", "combined", "wire_packed", "rl1_pieces", "rl1_head")}}
        modes = {"route_l1": {"CRDT_COMBINE": "0", "CRDT_ROUTE_L1": "1", "CRDT_RL1_SPLIT": "1"},
                 "route_l1_4": {"CRDT_COMBINE": "0", "CRDT_ROUTE_L1": "1", "CRDT_RL1_SPLIT": "4"},
                 "route_l1_head": {"CRDT_COMBINE": "0", "CRDT_ROUTE_L1": "2", "CRDT_RL1_SPLIT": "1"},
                 "combine": {"CRDT_COMBINE": "2", "CRDT_ROUTE_L1": "1"},
                 "route": {"CRDT_COMBINE": "0", "CRDT_ROUTE_L1": "0"}}
        saved = {k: os.environ.get(k) for k in ("CRDT_COMBINE", "CRDT_ROUTE_L1", "CRDT_RL1_SPLIT")}
        for name, env in modes.items():
            os.environ.update(env)
            reset()
            barrier()
            ts = time.perf_counter()
            r5 = step()
            barrier()
            ms5 = all_max(time.perf_counter() - ts) * 1e3
            p5 = table.last_plan()
            assert r5["status"] == 0 and r5["canonical_lt"] == res["canonical_lt"], (name, r5, res)
            route_ab[name] = {"ms": round(ms5, 3), "value": round(total_records / (ms5 / 1e3), 1),
                              "route_l1": p5["route_l1"], "combined": p5["combined"], "rl1_pieces": p5["rl1_pieces"],
                              "rl1_head": p5["rl1_head"]}
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    # ---- pre-sharded figure (N > 1): every rank already holds exactly what it owns
    presharded = None
    if world > 1 and args.config == "fanin" and not args.no_presharded:
        del wl["home"], src, cols
        torch.cuda.empty_cache()
        pw = gen_fanin(total=args.records, R=args.replicas, K=args.keys, n_local=args.local, s=args.zipf,
                       device=dev, order=args.order, rank=rank, world=world, route=False,
                       millis_span=args.millis_span)
        po = pw["owned"]
        cols = (po["key"], po["lt"], po["rank"], po["val"], pw["owned_offsets"])
        table.set_presharded(True)
        for _ in range(max(1, args.warmup)):
            reset()
            step()
        p_ms, p_sum, p_res = timed_run(args.steps)
        assert p_res["status"] == 0 and p_res["canonical_lt"] == res["canonical_lt"], (p_res, res)
        pm_ = float(np.mean(p_ms))
        presharded = {"value": round(total_records / (pm_ / 1e3), 1), "unit": "records/s",
                      "ms_per_step": round(pm_, 3), "step_ms_all": [round(x, 3) for x in p_ms],
                      "what": "same job, every record already on its owner (crdt_set_presharded): no record "
                              "exchange, only the clock collectives"}
        table.set_presharded(False)

    # ---- CPU baselines (rank 0, N = 1): the C restatement of the reference algorithm.
    # cpu_baseline: the faithful port on ONE thread (the reference is a single Dart isolate: its
    # recordMap() copy, clock reads, recv and winner loops all run on one core); cpu_baseline_copy16:
    # the same with only the map copy spread over 16 threads; cpu_baseline_omp: the optimised port
    if rank == 0 and world == 1 and not args.no_cpu:
        if job:                        # the census merged with win flags: redo the timed path's merge
            reset()
            step()
            torch.cuda.synchronize()
        cpu = cpu_baseline(wl, args.cpu_seconds, args.cpu_changesets, threads=1)
        if not args.no_cpu_copy16:
            cpu16 = cpu_baseline(wl, args.cpu_seconds, args.cpu_changesets)
        cpu_omp, parity = cpu_baseline_omp(wl, args.cpu_seconds, table)
    pcie = None
    if rank == 0 and world == 1 and not args.no_pcie and not wl.get("per_call"):
        pcie = host_input_rate(table, wl, reset)

    n = world
    out = {
        "metric": "merged records/sec (node) + % HBM roofline, 1B records x 1024 replicas",
        "value": round(value, 1), "unit": "records/s", "n_gpus": n, "steps": K,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
        "config": {"workload": workload, "records": total_records, "replicas": R,
                   "parallelism": f"keyshard{n}-routed" if world > 1 else "single", "merge_path": path,
                   "row_bytes": row_bytes,
                   "step_ms_all": [round(x, 3) for x in step_ms]},
        "roofline": roofline, "job": job, "cpu_baseline": cpu, "cpu_baseline_copy16": cpu16,
        "cpu_baseline_omp": cpu_omp, "host_nproc": os.cpu_count(), "parity": parity,
        "pcie_inclusive": pcie, "presharded": presharded, "route_ab": route_ab, "route_tune": route_tune, "placement": placement, "with_win_flags": with_flags,
        "gpu_clocks": gpu_clocks,
        "breakdown_ms": {"scan": round(tsum.get("scan_ms", 0) / K, 3),
                         "clock_verify_resolve": round(tsum.get("clock_ms", 0) / K, 3),
                         "route": round(tsum.get("route_ms", 0) / K, 3),
                         "apply_kernels_est": round(avg_launch_us * launches_per_step / 1e3, 3),
                         "apply_launches": launches_per_step,
                         "device_total": round(tsum.get("total_ms", 0) / K, 3)},
    }
    beat.stop()
    if world > 1:
        # the bytes this rank handed its peers per timed step (crdt_timing.sent_bytes), max over the ranks
        out["exchange"] = {"bytes_per_rank_per_step": int(all_max(tsum.get("sent_bytes", 0) / K)),
                           "plan": {k: v for k, v in plan.items()          # (the timed steps' way)
                                    if k in ("route_l1", "rl1_head", "combined", "rl1_pieces")}}
    if rank == 0:
        print(json.dumps(out), flush=True)
    table.close()
    if parity is not None and not parity["equal"]:
        log(f"PARITY FAILURE against the CPU oracle: {parity}")
        sys.exit(3)
    if world > 1:
        dist.destroy_process_group()


def make_workload(args, dev, rank, world, census):
    """The configuration's synthetic workload on this rank (BASELINE.json configs; crdt_amd/workload.py)."""
    from crdt_amd.workload import gen_cfg2, gen_cfg3, gen_cfg5, gen_fanin
    if args.config == "fanin":
        wl = gen_fanin(total=args.records, R=args.replicas, K=args.keys, n_local=args.local, s=args.zipf,
                       device=dev, order=args.order, rank=rank, world=world, route=world > 1, census=census,
                       millis_span=args.millis_span)
        workload = (f"fanin: {wl['total']:,} records = {wl['R']} replicas x {wl['n_per_replica']:,}, "
                    f"Zipf({args.zipf}) keys over 2^{int(np.log2(args.keys))} ids (unique per replica, "
                    f"{args.order} order), local map 2^{int(np.log2(args.local))} keys")
        if args.millis_span != 1 << 16:
            workload += f", clocks over {args.millis_span:,} ms"
        if world > 1:
            workload += (f"; replica j arrives whole on rank j % {world}, keys owned by rank key % {world}, "
                         f"records routed to their owner inside the step (one grouped all-to-all per step)")
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
        wl = gen_cfg5(device=dev, rank=rank, world=world)
        workload = ("cfg5 streaming: 100M-key table, 100 deltas x 10M records, one merge call per delta "
                    "(advancing wall), 10% tombstones, peers 1..16")
        if world > 1:
            workload += (f"; every delta split into {world} contiguous parts (part r on rank r), keys owned by "
                         f"rank key % {world}: one collective merge per delta routes the records to their owners")
    return wl, workload


def pmc_profile(args, path, world):
    """The committed rocprofv3 --pmc summary (PMC_FILE) when it was taken on this exact command."""
    if not os.path.exists(PMC_FILE) or args.config != "fanin" or world != 1:
        return None
    try:
        pm = json.load(open(PMC_FILE))
    except Exception:  # noqa: BLE001
        return None
    if pm.get("command_args") != pmc_args(args) or pm.get("merge_path") != path:
        return None
    return pm


def pmc_kernel(args, path, name, world):
    """Per-step HBM bytes of the kernel whose name starts with ``name`` in the PMC summary."""
    pm = pmc_profile(args, path, world)
    if not pm:
        return None
    for k, v in pm.get("kernels", {}).items():
        if k.startswith(name + "<") or k == name:
            return dict(v, source=os.path.relpath(PMC_FILE, ROOT) + f" [{k}]")
    return None


def pmc_args(args) -> list:
    """The arguments that define the workload a committed PMC profile must match."""
    out = [args.config, args.records, args.replicas, args.keys, args.local, args.zipf, args.order, args.path,
           bool(args.exact_counts)]
    if args.millis_span != 1 << 16:
        out.append(args.millis_span)
    return out


def cpu_baseline(wl, budget_s, n_changesets=64, threads=None):
    """Times oracle/merge_oracle.c in faithful mode — the reference algorithm: a full recordMap()
    copy of the map per merge (map_crdt.dart:43, on ``threads`` threads: the only unordered part),
    the recv loop with a clock read per record (hlc.dart:82) and the winner loop, sequential — on the
    first ``n_changesets`` changesets of the same workload (stopping early past ~budget_s x 4,
    threads=1: past ~budget_s), in blocks of changesets whose rates give the spread."""
    import torch
    from oracle.oracle_c import OracleTable
    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(os.cpu_count() or 1, 16)
    block = 8 if threads > 1 else 2
    limit = 4 * budget_s if threads > 1 else budget_s
    loc = wl["local"]
    cap = wl["capacity"]
    t = OracleTable(cap, 0, wl["c0"])
    t.put_rows(loc["slot"].cpu().numpy().astype(np.uint32), loc["lt"].cpu().numpy(),
               loc["rank"].cpu().numpy().astype(np.uint32), loc["val"].cpu().numpy().astype(np.uint32),
               loc["mod"].cpu().numpy())
    offs = wl["owned_offsets"]
    own = wl["owned"]
    want = min(n_changesets, wl["R"])
    done, recs, el, blocks = 0, 0, 0.0, []
    while done < want and el < limit:
        j1 = min(done + block, want)
        b, e = int(offs[done]), int(offs[j1])
        cols = [own[k][b:e].cpu().numpy() for k in ("key", "lt", "rank", "val")]
        sub = (offs[done:j1 + 1] - offs[done]).astype(np.uint64)
        wall = int(wl["walls"][done]) if wl.get("per_call") else wl["wall"]
        ts = time.perf_counter()
        res, _ = t.merge(cols[0].astype(np.uint32), cols[1], cols[2].astype(np.uint32),
                         cols[3].astype(np.uint32), sub, wall, faithful=threads, want_flags=False)
        dt = time.perf_counter() - ts
        assert res.status == 0
        el += dt
        blocks.append((e - b) / dt)
        done = j1
        recs += e - b
    del t
    torch.cuda.synchronize()
    return {"value": round(recs / el, 1), "unit": "records/s", "cores": threads, "kind": "port",
            "spread": {"min": round(min(blocks), 1), "median": round(float(np.median(blocks)), 1),
                       "max": round(max(blocks), 1), "blocks": len(blocks), "changesets_per_block": block},
            "sample": f"first {done} of {wl['R']} changesets ({recs:,} records, {100 * recs / wl['total']:.1f} % of "
                      f"the batch) merged into the full {cap:,}-row map by oracle/merge_oracle.c in faithful "
                      f"mode: one full map copy per merge (map_crdt.dart:43) on {threads} thread"
                      f"{'s' if threads > 1 else ''}, one clock read per record (hlc.dart:82) and the recv / "
                      f"winner loops on one thread, {el:.1f}s; host nproc {os.cpu_count()}"}


def cpu_baseline_omp(wl, budget_s, table=None, keep=False):
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
    kept = t if keep and done == wl["R"] else None
    del t
    torch.cuda.synchronize()
    base = {"value": round(recs / el, 1), "unit": "records/s", "cores": threads, "kind": "port",
            "sample": f"first {done} of {wl['R']} changesets ({recs:,} records) merged by oracle/merge_omp.c "
                      f"(parallel per-changeset max / apply, exact recv loop only on flagged changesets), "
                      f"{threads} OpenMP threads, {el:.1f}s",
            "threads_why": "OMP_NUM_THREADS (16 on the GPU box: one GPU's share of its host; os.cpu_count() reports "
                           "the whole machine, whose cores serve every GPU of the node), else min(cpu_count, 16)"}
    if keep:
        return base, parity, kept
    return base, parity


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


DIGEST_BLOCK = 1 << 20          # slots per parity digest word
_DIG_P = [np.uint64(x) for x in (0x9E3779B97F4A7C15, 0xC2B2AE3D27D4EB4F, 0x165667B19E3779F9,
                                 0xD6E8FEB86659FD93, 0xFF51AFD7ED558CCD)]


def row_digests(lt, rank, val, mod, slot0: int) -> np.ndarray:
    """One 64-bit word per DIGEST_BLOCK slots (slot0 a multiple of it): the wrapping sum over the
    block of a mix of (slot, lt, rank, val, mod) — equal blocks give equal words, and a row that
    differs in any field (or sits at another slot) changes its block's word."""
    n = len(lt)
    with np.errstate(over="ignore"):
        slot = np.arange(slot0, slot0 + n, dtype=np.uint64)
        rv = (np.asarray(rank).astype(np.uint64) << np.uint64(32)) | np.asarray(val).astype(np.uint64)
        h = (np.asarray(lt).view(np.uint64) * _DIG_P[0]) ^ (np.asarray(mod).view(np.uint64) * _DIG_P[1])
        h ^= rv * _DIG_P[2]
        h ^= slot * _DIG_P[3]
        h ^= h >> np.uint64(29)
        h *= _DIG_P[4]
        h ^= h >> np.uint64(32)
    starts = np.arange(0, n, DIGEST_BLOCK)
    return np.add.reduceat(h, starts) if n else np.zeros(0, np.uint64)


def shard_digests(table, cap: int, chunk: int = 1 << 25) -> np.ndarray:
    """row_digests of this rank's table, slots [0, cap)."""
    out = []
    for b in range(0, cap, chunk):
        e = min(b + chunk, cap)
        lt, rk, val, mod = table.read_rows(np.arange(b, e, dtype=np.uint32))
        out.append(row_digests(lt, rk, val, mod, b))
    return np.concatenate(out) if out else np.zeros(0, np.uint64)


def shard_parity(oracle, got, world: int) -> dict:
    """Every rank's shard digests (``got``: (rank, digests, canonical) per rank) against the same
    digests of the oracle's rows key % world == rank at slot key // world."""
    from oracle.oracle_c import new_table
    ts = time.perf_counter()
    K = len(oracle.rows)
    bad_blocks, canon_bad, blocks = 0, 0, 0
    for r, dig, canon in got:
        sh = oracle.rows[r::world]
        cap = len(dig) and -(-K // world)
        if len(sh) < cap:                              # slots past the last key: never-written fill
            sh = np.concatenate([sh, new_table(cap - len(sh))])
        want = row_digests(sh["lt"], sh["rank"], sh["val"], sh["mod"], 0)
        d = np.asarray(dig, np.uint64)
        blocks += len(want)
        bad_blocks += int(np.count_nonzero(d != want)) if len(d) == len(want) else len(want)
        canon_bad += int(canon != oracle.canonical)
    return {"rows": K, "shards": world, "digest_blocks": blocks, "blocks_differing": bad_blocks,
            "canonical_equal": canon_bad == 0, "equal": bad_blocks == 0 and canon_bad == 0,
            "against": "oracle/merge_omp.c final state of the unsharded batch, per-shard digests "
                       f"(one 64-bit word per {DIGEST_BLOCK} slots: bench.row_digests)",
            "seconds": round(time.perf_counter() - ts, 1)}


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
