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

static PyMethodDef fc_methods[] = {
    {"bind", fc_bind, METH_VARARGS, "bind(address of pv_verify_batch)"},
    {"verify", fc_verify, METH_VARARGS, "verify(blob, offsets, pks, bits) -> pv_verify_batch's return code"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef fc_module = {PyModuleDef_HEAD_INIT, "_fastcall", NULL, -1, fc_methods,
                                       NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__fastcall(void) { return PyModule_Create(&fc_module); }
