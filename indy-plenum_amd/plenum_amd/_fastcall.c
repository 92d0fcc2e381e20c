/* CPython binding of pv_verify_batch for small host-buffer calls (Plenum's feed-point quotas and
 * verifySignature singletons, stp_core/crypto/nacl_wrappers.py:232-242 -> Verifier.verify): the
 * buffer protocol instead of ctypes pointer marshalling (~2 us per numpy array on the host), the GIL
 * released around the call. Same C ABI entry point and same validation as plenum_amd/_native.py's
 * ctypes path, which stays as the fallback when this module is not built. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

typedef int (*pv_verify_batch_fn)(const uint8_t*, const uint64_t*, uint64_t, const uint8_t*, uint8_t*);
static pv_verify_batch_fn g_verify = NULL;

/* bind(address): the address of pv_verify_batch in the already loaded libplenum_verify.so */
static PyObject* fc_bind(PyObject* self, PyObject* args) {
    unsigned long long addr;
    (void)self;
    if (!PyArg_ParseTuple(args, "K", &addr)) return NULL;
    g_verify = (pv_verify_batch_fn)(uintptr_t)addr;
    Py_RETURN_NONE;
}

/* verify(blob, offsets, pks, bits) -> rc: C-contiguous buffers of n + 1 uint64 offsets into blob,
 * n x 32 key bytes and ceil(n / 8) writable verdict bytes (LSB-first). */
static PyObject* fc_verify(PyObject* self, PyObject* args) {
    PyObject *ob, *oo, *op, *ov;
    Py_buffer b, o, p, v;
    int rc = -1;
    (void)self;
    if (!g_verify) {
        PyErr_SetString(PyExc_RuntimeError, "_fastcall.bind() was not called");
        return NULL;
    }
    if (!PyArg_ParseTuple(args, "OOOO", &ob, &oo, &op, &ov)) return NULL;
    if (PyObject_GetBuffer(ob, &b, PyBUF_C_CONTIGUOUS) < 0) return NULL;
    if (PyObject_GetBuffer(oo, &o, PyBUF_C_CONTIGUOUS) < 0) goto rel_b;
    if (PyObject_GetBuffer(op, &p, PyBUF_C_CONTIGUOUS) < 0) goto rel_o;
    if (PyObject_GetBuffer(ov, &v, PyBUF_C_CONTIGUOUS | PyBUF_WRITABLE) < 0) goto rel_p;
    {
        const uint64_t n = o.len >= 16 ? (uint64_t)(o.len / 8) - 1 : 0;
        const uint64_t* off = (const uint64_t*)o.buf;
        if (o.len % 8 || n == 0 || (uint64_t)p.len < 32 * n || (uint64_t)v.len < (n + 7) / 8 ||
            off[n] > (uint64_t)b.len) {
            PyErr_SetString(PyExc_ValueError, "verify: inconsistent blob / offsets / keys / verdict sizes");
        } else {
            Py_BEGIN_ALLOW_THREADS
            rc = g_verify((const uint8_t*)b.buf, off, n, (const uint8_t*)p.buf, (uint8_t*)v.buf);
            Py_END_ALLOW_THREADS
        }
    }
    PyBuffer_Release(&v);
rel_p:
    PyBuffer_Release(&p);
rel_o:
    PyBuffer_Release(&o);
rel_b:
    PyBuffer_Release(&b);
    if (PyErr_Occurred()) return NULL;
    return PyLong_FromLong(rc);
}

/* verify_one(pk, sm) -> rc < 0 (the library's error code) or the verdict (0 / 1): ONE (32-byte key,
 * signature || message) pair from two bytes-like objects, with no arrays built around them -- the
 * unbatched drop-in's verifySignature singleton (nacl_wrappers.py:232-242). */
static PyObject* fc_verify_one(PyObject* self, PyObject* args) {
    Py_buffer k, m;
    int rc = -1;
    (void)self;
    if (!g_verify) {
        PyErr_SetString(PyExc_RuntimeError, "_fastcall.bind() was not called");
        return NULL;
    }
    if (!PyArg_ParseTuple(args, "y*y*", &k, &m)) return NULL;
    if (k.len != 32) {
        PyErr_SetString(PyExc_ValueError, "verify_one: the key must be 32 bytes");
    } else {
        static const uint8_t empty[1] = {0};
        const uint64_t off[2] = {0, (uint64_t)m.len};
        uint8_t bit = 0;
        Py_BEGIN_ALLOW_THREADS
        rc = g_verify(m.len ? (const uint8_t*)m.buf : empty, off, 1, (const uint8_t*)k.buf, &bit);
        Py_END_ALLOW_THREADS
        if (rc == 0) rc = bit & 1;
    }
    PyBuffer_Release(&m);
    PyBuffer_Release(&k);
    if (PyErr_Occurred()) return NULL;
    return PyLong_FromLong(rc);
}

/* finish_single(verified, results, a, b, keys_hex, sig_lines, sig_off, pair_off, pair_name, names):
 * plenum_amd/wire.py's per-request finish of device-verified single-signature requests a..b-1, in
 * request order, as ReqAuthenticator.authenticate leaves them (plenum/server/req_authenticator.py:
 * 31-50): key = Request.digest (64 hex digits, line i of keys_hex), sig = the signature text (line
 * pair_off[i] of sig_lines); if verified[key] exists with the same 'signature' its 'identifiers'
 * are the result, else verified[key] = {'signature': sig, 'identifiers': {identifier}} and that set
 * is. `verified` must be an exact dict and `results` a list (the caller checks). Exceptions raised
 * by an existing entry's lookup or comparison propagate, as they do from the Python loop. */
static PyObject* fc_finish_single(PyObject* self, PyObject* args) {
    PyObject *verified, *results, *names, *okh, *osl, *oso, *opo, *opn;
    Py_ssize_t a, b;
    Py_buffer kh, sl, so, po, pn;
    PyObject* ret = NULL;
    PyObject *k_sig = NULL, *k_ids = NULL;
    (void)self;
    if (!PyArg_ParseTuple(args, "O!O!nnOOOOOO!", &PyDict_Type, &verified, &PyList_Type, &results, &a, &b, &okh,
                          &osl, &oso, &opo, &opn, &PyList_Type, &names))
        return NULL;
    if (PyObject_GetBuffer(okh, &kh, PyBUF_C_CONTIGUOUS) < 0) return NULL;
    if (PyObject_GetBuffer(osl, &sl, PyBUF_C_CONTIGUOUS) < 0) goto r_kh;
    if (PyObject_GetBuffer(oso, &so, PyBUF_C_CONTIGUOUS) < 0) goto r_sl;
    if (PyObject_GetBuffer(opo, &po, PyBUF_C_CONTIGUOUS) < 0) goto r_so;
    if (PyObject_GetBuffer(opn, &pn, PyBUF_C_CONTIGUOUS) < 0) goto r_po;
    {
        const char* keys = (const char*)kh.buf;
        const char* lines = (const char*)sl.buf;
        const uint64_t* soff = (const uint64_t*)so.buf;
        const uint64_t* poff = (const uint64_t*)po.buf;
        const uint32_t* pname = (const uint32_t*)pn.buf;
        const Py_ssize_t n_pairs = so.len / 8 - 1, n_names = PyList_GET_SIZE(names);
        if (a < 0 || b < a || b > PyList_GET_SIZE(results) || kh.len < 65 * b || po.len < 8 * (b + 1) ||
            so.len < 8 || so.len % 8 || pn.len < 4 * n_pairs) {
            PyErr_SetString(PyExc_ValueError, "finish_single: inconsistent plan buffers");
            goto done;
        }
        k_sig = PyUnicode_InternFromString("signature");
        k_ids = PyUnicode_InternFromString("identifiers");
        if (!k_sig || !k_ids) goto done;
        for (Py_ssize_t i = a; i < b; i++) {
            const Py_ssize_t p = (Py_ssize_t)poff[i];
            if (p < 0 || p >= n_pairs || pname[p] >= (uint64_t)n_names ||
                (Py_ssize_t)(soff[p + 1] + p + 1) > sl.len || soff[p + 1] < soff[p]) {
                PyErr_SetString(PyExc_ValueError, "finish_single: pair index out of range");
                goto done;
            }
            const char* kp = keys + 65 * i;
            Py_ssize_t kl = 0;
            while (kl < 64 && kp[kl] != '\n') kl++;
            PyObject* key = PyUnicode_DecodeASCII(kp, kl, NULL);
            if (!key) goto done;
            PyObject* sig = PyUnicode_DecodeASCII(lines + soff[p] + p, (Py_ssize_t)(soff[p + 1] - soff[p]), NULL);
            if (!sig) { Py_DECREF(key); goto done; }
            PyObject* seen = PyDict_GetItemWithError(verified, key);  /* borrowed */
            PyObject* res = NULL;
            if (seen) {
                Py_INCREF(seen);
                PyObject* old = PyObject_GetItem(seen, k_sig);
                int same = old ? PyObject_RichCompareBool(old, sig, Py_EQ) : -1;
                Py_XDECREF(old);
                if (same > 0) res = PyObject_GetItem(seen, k_ids);
                Py_DECREF(seen);
                if (same < 0 || (same > 0 && !res)) { Py_DECREF(key); Py_DECREF(sig); goto done; }
            } else if (PyErr_Occurred()) {
                Py_DECREF(key); Py_DECREF(sig); goto done;
            }
            if (!res) {
                PyObject* ids = PySet_New(NULL);
                PyObject* ent = PyDict_New();
                if (!ids || !ent || PySet_Add(ids, PyList_GET_ITEM(names, pname[p])) < 0 ||
                    PyDict_SetItem(ent, k_sig, sig) < 0 || PyDict_SetItem(ent, k_ids, ids) < 0 ||
                    PyDict_SetItem(verified, key, ent) < 0) {
                    Py_XDECREF(ids); Py_XDECREF(ent); Py_DECREF(key); Py_DECREF(sig); goto done;
                }
                Py_DECREF(ent);
                res = ids;
            }
            Py_DECREF(key);
            Py_DECREF(sig);
            PyList_SetItem(results, i, res);  /* steals res, releases the previous item */
        }
        ret = Py_None;
        Py_INCREF(ret);
    }
done:
    Py_XDECREF(k_sig);
    Py_XDECREF(k_ids);
    PyBuffer_Release(&pn);
r_po:
    PyBuffer_Release(&po);
r_so:
    PyBuffer_Release(&so);
r_sl:
    PyBuffer_Release(&sl);
r_kh:
    PyBuffer_Release(&kh);
    return ret;
}

static PyMethodDef fc_methods[] = {
    {"bind", fc_bind, METH_VARARGS, "bind(address of pv_verify_batch)"},
    {"verify", fc_verify, METH_VARARGS, "verify(blob, offsets, pks, bits) -> pv_verify_batch's return code"},
    {"verify_one", fc_verify_one, METH_VARARGS, "verify_one(pk, sm) -> error code < 0, or the verdict 0 / 1"},
    {"finish_single", fc_finish_single, METH_VARARGS,
     "finish_single(verified, results, a, b, keys_hex, sig_lines, sig_off, pair_off, pair_name, names)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef fc_module = {PyModuleDef_HEAD_INIT, "_fastcall", NULL, -1, fc_methods,
                                       NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__fastcall(void) { return PyModule_Create(&fc_module); }
