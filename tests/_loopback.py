"""A loopback crdt_comm_ops (device memory) for rank 0 of G ranks that all hold rank 0's data: the
all-gather repeats rank 0's row, the reductions keep its words, and the all-to-all hands back, from each
peer d, a device copy (hipMemcpyAsync on the ctx stream) of exactly the bytes rank 0 sends d.  It drives
the library's device-memory collective path (the one RCCL takes: no host synchronisation inside the
collectives) on one GPU; tools/route_probe.py times it, tests/test_gpu_parity.py checks that every way of
routing leaves the same rows under it.  Test / tool infrastructure."""
import ctypes

from crdt_amd import _capi

hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipEventCreate.argtypes = [ctypes.c_void_p]
hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]
D2D = 3


class LoopbackComm:
    """crdt_comm_ops (device memory) for rank 0 of G ranks that all hold rank 0's data."""

    def __init__(self, G):
        self.G = G
        self.error = None
        self.evs = []                                  # (start, end) events around each record exchange
        self.sent = 0                                  # bytes rank 0 sent its peers (all exchanges)

    def _event(self):
        e = ctypes.c_void_p()
        assert hip.hipEventCreate(ctypes.byref(e)) == 0
        return e

    def exchange_ms(self):
        ms, tot = ctypes.c_float(), 0.0
        for a, b in self.evs:
            hip.hipEventSynchronize(b)
            hip.hipEventElapsedTime(ctypes.byref(ms), a, b)
            tot += ms.value
        self.evs = []
        return tot

    def exchange_bytes(self):
        b, self.sent = self.sent, 0
        return b

    def ops(self):
        G = self

        def guard(fn):
            def call(*a):
                try:
                    return fn(*a)
                except Exception as e:  # noqa: BLE001
                    G.error = e
                    return 1
            return call

        def _ar(user, words, n, op, stream):
            return 0                                   # identical words on every rank

        def _ag(user, send, recv, n, stream):
            for r in range(G.G):
                assert hip.hipMemcpyAsync(recv + r * n * 8, send, n * 8, D2D, stream) == 0
            return 0

        def _a2a(user, n_cols, send, recv, eb, sc, sd, rc, rd, stream):
            nbytes = sum(sc[d] * eb[k] for d in range(G.G) for k in range(n_cols))
            G.sent += nbytes
            big = nbytes > (1 << 20)
            if big:
                a, b = G._event(), G._event()
                hip.hipEventRecord(a, stream)
            for d in range(G.G):
                for k in range(n_cols):
                    nb = min(sc[d], rc[d]) * eb[k]
                    if nb:
                        assert hip.hipMemcpyAsync(recv[k] + rd[d] * eb[k], send[k] + sd[d] * eb[k], nb, D2D,
                                                  stream) == 0
            if big:
                hip.hipEventRecord(b, stream)
                G.evs.append((a, b))
            return 0

        self._cbs = (_capi.ALL_REDUCE_FN(guard(_ar)), _capi.ALL_GATHER_FN(guard(_ag)),
                     _capi.ALL_TO_ALL_FN(guard(_a2a)))
        return _capi.CrdtCommOps(None, _capi.CRDT_MEM_DEVICE, 0, *self._cbs)


