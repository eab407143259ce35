"""Exports golden cases of merge_golden.npz / .json to tests/golden/abi_cases.bin, the flat
little-endian file tests/c/abi_golden.c reads (a C host with no Python or torch in it).

Layout: "CRDTABI1", u32 n_cases; per case: char name[32]; u32 n_ids, n_local, local_rank, R;
u64 n; i64 c0, wall; u32 has_millis, pad; local i64 lt[n_local], u32 rank[n_local],
u32 val[n_local], i64 mod[n_local]; batch u32 key[n], i64 lt[n], u32 rank[n], u32 val[n],
u64 offsets[R + 1], (i64 millis[n] if has_millis); expected i32 status, u32 n_stored,
u32 exc_changeset, u32 pad, u64 exc_index, i64 canonical, i64 drift, i64 counter,
u64 n_present, u64 n_won; u8 exists[n_ids], i64 lt[n_ids], u32 rank[n_ids], u32 val[n_ids],
i64 mod[n_ids], u8 flags[n].   Re-run:  python tests/golden/export_abi_cases.py
"""
import json
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = ["r4_ties", "dup_node", "explicit_millis", "send_overflow", "r8_tombstones"]


def main():
    arr = np.load(os.path.join(HERE, "merge_golden.npz"))
    meta = json.load(open(os.path.join(HERE, "merge_golden.json")))
    out = [b"CRDTABI1", struct.pack("<I", len(CASES))]
    for name in CASES:
        m, p = meta[name], name + "__"
        g = lambda f, dt: np.ascontiguousarray(arr[p + f], dtype=dt).tobytes()  # noqa: E731
        offs = arr[p + "offsets"]
        R, n = len(offs) - 1, int(offs[-1])
        has_millis = (p + "millis") in arr.files
        out.append(name.encode().ljust(32, b"\0"))
        out.append(struct.pack("<IIIIQqqII", m["n_ids"], m["n_local"], m["local_rank"], R, n, m["c0"], m["wall"],
                               int(has_millis), 0))
        out += [g("local_lt", "<i8"), g("local_rank", "<u4"), g("local_val", "<u4"), g("local_mod", "<i8")]
        out += [g("key", "<u4"), g("lt", "<i8"), g("rank", "<u4"), g("val", "<u4"), g("offsets", "<u8")]
        if has_millis:
            out.append(g("millis", "<i8"))
        e = m["expected"]
        out.append(struct.pack("<iIIIQqqqQQ", e["status"], e["n_stored"], e["exc_changeset"], 0, e["exc_index"],
                               e["canonical_lt"], e["drift_ms"], e["counter"], e["n_present"], e["n_won"]))
        out += [g("exp_exists", "<u1"), g("exp_lt", "<i8"), g("exp_rank", "<u4"), g("exp_val", "<u4"),
                g("exp_mod", "<i8"), g("exp_flags", "<u1")]
    with open(os.path.join(HERE, "abi_cases.bin"), "wb") as f:
        f.write(b"".join(out))
    print(f"{len(CASES)} cases, {sum(len(x) for x in out)} bytes")


if __name__ == "__main__":
    main()
