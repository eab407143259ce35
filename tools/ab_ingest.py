import sys,time,os,json
R=os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0,R); sys.path.insert(0,os.path.join(R,'tools'))
from ingest_bench import make_doc
from crdt_amd import hostlib
from crdt_amd.intern import KeyIndex
doc=make_doc(1000000)
res={}
for rep in range(5):
    for mode in ("0","1"):
        os.environ["CRDT_HOST_PREFAULT"]=mode
        k=KeyIndex(); t=time.perf_counter(); d=hostlib.decode(doc,k.native); dt=time.perf_counter()-t
        res.setdefault(mode,[]).append(round(dt*1e3,1))
        del d,k
print(json.dumps({"prefault_off_ms":res["0"],"prefault_on_ms":res["1"]}))
