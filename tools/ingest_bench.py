#!/usr/bin/env python3
"""Host-ingest throughput: CrdtJson.decode of an N-record document by the native
decoder (libcrdt_host.so) vs the Python restatement, and (with --gpu) MapCrdt.mergeJson
end to end on the GPU both ways, then the export (MapCrdt.toJson of the merged map:
device compaction + native encode vs the Python restatement).  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from crdt_amd import hostlib  # noqa: E402
from crdt_amd.crdt_json import CrdtJson  # noqa: E402
from crdt_amd.hlc import Hlc  # noqa: E402
from crdt_amd.intern import KeyIndex  # noqa: E402


def make_doc(n, seed=1):
    rng = np.random.default_rng(seed)
    base = 1_735_689_600_000
    ms = base + rng.integers(0, 1 << 20, n)
    cnt = rng.integers(0, 16, n)
    lt = (ms << 16) + cnt
    nodes = [f"peer{i:03d}" for i in range(16)]
    node = rng.integers(0, 16, n).astype(np.uint32)
    hlcs = hostlib.hlc_strings(lt, node, nodes)
    vals = rng.integers(0, 1 << 30, n)
    parts = [f'"key{i:08d}":{{"hlc":"{hlcs[i]}","value":{int(vals[i]) if i % 10 else "null"}}}' for i in range(n)]
    return "{" + ",".join(parts) + "}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1_000_000)
    ap.add_argument("--gpu", action="store_true")
    a = ap.parse_args()
    doc = make_doc(a.records)
    out = {"records": a.records, "doc_mb": round(len(doc) / 1e6, 1)}
    t = time.perf_counter()
    keys = KeyIndex()
    dec = hostlib.decode(doc, keys.native)
    out["native_decode_s"] = round(time.perf_counter() - t, 3)
    assert len(dec["key_id"]) == a.records
    t = time.perf_counter()
    CrdtJson.decode(doc, Hlc(0, 0, "local"), millis=1_735_689_600_000)
    out["python_decode_s"] = round(time.perf_counter() - t, 3)
    out["native_decode_rps"] = round(a.records / out["native_decode_s"])
    out["python_decode_rps"] = round(a.records / out["python_decode_s"])
    if a.gpu:
        from crdt_amd import MapCrdt
        wall = 1_735_689_600_000 + (1 << 20) + 1000
        w = MapCrdt("local", capacity=a.records + 16)       # warm-up: code objects, host threads
        w.mergeJson(doc, wall=wall)
        del w
        for mode in ("native", "python"):
            c = MapCrdt("local", capacity=a.records + 16)
            if mode == "python":
                c._native_ingest = lambda: False
            c.put("warm", 1, wall=wall)
            t = time.perf_counter()
            c.mergeJson(doc, wall=wall)
            out[f"mergeJson_{mode}_s"] = round(time.perf_counter() - t, 3)
            assert c.last_ingest == mode
            out[f"mergeJson_{mode}_rps"] = round(a.records / out[f"mergeJson_{mode}_s"])
            # export of the merged map: raw input spans (native ingest) or Python values (python)
            from crdt_amd.crdt import Crdt
            t = time.perf_counter()
            js = c.toJson()
            out[f"toJson_native_{mode}vals_s"] = round(time.perf_counter() - t, 3)
            assert c.last_export == "native"
            if mode == "native":
                t = time.perf_counter()                 # the same document again: every record loses
                c.mergeJson(doc, wall=wall)
                out["mergeJson_native_again_s"] = round(time.perf_counter() - t, 3)
                t = time.perf_counter()
                ref = Crdt.toJson(c)
                out["toJson_python_s"] = round(time.perf_counter() - t, 3)
                assert js == ref
                out["toJson_native_rps"] = round((a.records + 1) / out["toJson_native_nativevals_s"])
                out["toJson_python_rps"] = round((a.records + 1) / out["toJson_python_s"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
