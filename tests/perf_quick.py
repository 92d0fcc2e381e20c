"""Quick device-resident throughput probe (measurement helper; under tests/ because it signs with
the libsodium loader of oracle/; bench.py is the contract)."""
import ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "indy-plenum_amd"), os.path.join(ROOT, "tests")]
from plenum_amd import _native
from oracle.libsodium_ref import LibSodium
ls = LibSodium()
n_unique = int(os.environ.get("NU", "8192")); n = int(os.environ.get("N", str(1 << 20)))
rng = np.random.default_rng(1)
cases = []
for i in range(n_unique):
    pk, sk = ls.seed_keypair(rng.bytes(32))
    m = rng.bytes(299)
    cases.append((ls.sign_detached(m, sk) + m, pk))
reps = n // n_unique
blob = np.frombuffer(b"".join(sm for sm, _ in cases) * reps, np.uint8)
pks = np.frombuffer(b"".join(pk for _, pk in cases) * reps, np.uint8)
off = np.arange(n + 1, dtype=np.uint64) * 363
_native.ensure_device()
L = _native.lib()
def dalloc(b):
    p = ctypes.c_void_p(); _native.check(L.pv_dev_alloc(ctypes.byref(p), b), "alloc"); return p
d_blob = dalloc(blob.nbytes + 256); d_off = dalloc(off.nbytes); d_pk = dalloc(pks.nbytes); d_v = dalloc((n + 63) // 64 * 8)
L.pv_memcpy_h2d(d_blob, blob.ctypes.data, blob.nbytes); L.pv_memcpy_h2d(d_off, off.ctypes.data, off.nbytes); L.pv_memcpy_h2d(d_pk, pks.ctypes.data, pks.nbytes)
L.pv_set_timing(1)
rows = []
for it in range(int(os.environ.get("IT", "3"))):
    t = time.time()
    _native.check(L.pv_verify_batch_device(d_blob, d_off, n, d_pk, d_v, None), "verify")
    _native.check(L.pv_sync(), "sync")
    dt = time.time() - t
    st = (ctypes.c_double * 5)(); nl = ctypes.c_int()
    L.pv_stage_times(st, 5, ctypes.byref(nl)); L.pv_set_timing(1)
    v = np.zeros((n + 63) // 64, np.uint64); L.pv_memcpy_d2h(v.ctypes.data, d_v, v.nbytes)
    ok = int(np.unpackbits(v.view(np.uint8), bitorder="little")[:n].sum())
    row = {"n": n, "wall_s": round(dt, 4), "verifies_per_s": round(n / dt),
           **{k + "_ms": round(v, 3) for k, v in zip(_native.PV_STAGES, st)}, "valid": ok}
    rows.append(row)
    if os.environ.get("VERBOSE"):
        print(row, flush=True)
tail = rows[min(3, len(rows) - 1):]
med = {k: float(np.median([r[k] for r in tail])) for k in tail[0] if k.endswith("_ms")}
print({"lib": os.path.basename(_native.LIB_PATH), "iters": len(tail), "valid": rows[-1]["valid"],
       "sum_ms": round(sum(med.values()), 4), **{k: round(v, 4) for k, v in med.items()}}, flush=True)
