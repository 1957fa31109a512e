/* _hostfast: the per-call host work of a fold that Python does one object at
 * a time, in one C loop (CPython extension, host only).
 *
 * round_weak_f32(seq) -> bytes | None
 *   The reference multiplies a float32 layer by Python numbers
 *   (fed_avg_aggregator.py:32-41: `layer * n`, stall_aware_aggregation.py:57-63:
 *   `layer * n * s`).  Under NEP 50 a Python bool / int / float is a "weak"
 *   scalar: it is rounded to float32 first and the result stays float32.  For
 *   a sequence whose items are ALL exactly bool, int or float (no subclass,
 *   no numpy scalar) this returns the float32 roundings, native byte order,
 *   as bytes: float(v) rounded to nearest-even float32, which is numpy's
 *   np.float32(v) for every such value whose float64 conversion is exact
 *   (|int| < 2**53; every float).  Anything else -- another type, a larger
 *   int -- returns None and the caller takes the general numpy path
 *   (engine.result_dtype / engine.round_scalars), so results never depend on
 *   whether this module is present.
 *
 * alloc_bytes(n) -> (bytes, address): see below.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

static PyObject* round_weak_f32(PyObject* self, PyObject* arg) {
    (void)self;
    PyObject* seq = PySequence_Fast(arg, "round_weak_f32: expected a sequence");
    if (!seq) return NULL;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    PyObject** items = PySequence_Fast_ITEMS(seq);
    PyObject* out = PyBytes_FromStringAndSize(NULL, n * (Py_ssize_t)sizeof(float));
    if (!out) {
        Py_DECREF(seq);
        return NULL;
    }
    float* f = (float*)PyBytes_AS_STRING(out);
    const long long lim = 1LL << 53;
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* o = items[i];
        double d;
        if (PyFloat_CheckExact(o)) {
            d = PyFloat_AS_DOUBLE(o);
        } else if (PyLong_CheckExact(o) || PyBool_Check(o)) {
            int overflow = 0;
            const long long v = PyLong_AsLongLongAndOverflow(o, &overflow);
            if (overflow || v >= lim || v <= -lim) goto general;
            d = (double)v;
        } else {
            goto general;
        }
        f[i] = (float)d;
    }
    Py_DECREF(seq);
    return out;
general:
    Py_DECREF(seq);
    Py_DECREF(out);
    Py_RETURN_NONE;
}

/* alloc_bytes(n) -> (bytes, address)
 *   A new, uninitialised bytes object of n bytes and the address of its
 *   storage, for a native writer to fill (fedlesscan_amd/npz.py write_npz
 *   assembles the saved model with the threaded fa_pack) before the object is
 *   handed to anyone else. */
static PyObject* alloc_bytes(PyObject* self, PyObject* arg) {
    (void)self;
    const Py_ssize_t n = PyLong_AsSsize_t(arg);
    if (n < 0) {
        if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "alloc_bytes: negative size");
        return NULL;
    }
    PyObject* b = PyBytes_FromStringAndSize(NULL, n);
    if (!b) return NULL;
    PyObject* addr = PyLong_FromVoidPtr((void*)PyBytes_AS_STRING(b));
    if (!addr) {
        Py_DECREF(b);
        return NULL;
    }
    return Py_BuildValue("(NN)", b, addr);
}

static PyMethodDef methods[] = {
    {"alloc_bytes", alloc_bytes, METH_O, "(uninitialised bytes of n bytes, its storage address)"},
    {"round_weak_f32", round_weak_f32, METH_O,
     "float32 roundings of a sequence of Python bool/int/float as bytes, or None for anything else"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_hostfast", NULL, -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__hostfast(void) { return PyModule_Create(&module); }
