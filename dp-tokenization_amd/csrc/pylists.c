/* dptok._pylists: the host path's last step -- CSR ids (int32 ids, uint64 offsets, int32 statuses) into
 * the drop-in's Python shape, a list of (List[int], status) per string -- in one pass of C.
 *
 * The Python form (ids.tolist() and a slice per string) spends ~20 ns per id allocating an int object
 * and copying it into a slice: ~50 ms for cfg2's 4096 x 256-byte batch of 856k ids, 20x the GPU call.
 * Here every id's int object comes from a per-process cache indexed by id (ids are vocabulary indices:
 * one object each, referenced, never reallocated), and each string's list is filled directly.
 *
 * Reference shape: tokenizer_utils.py:66-80 (dp_tokenize returns List[int] per string).  Pure data
 * marshalling: no tokenization happens here. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

static PyObject **g_cache = NULL;   /* g_cache[id]: the int object of id (one reference held here) */
static Py_ssize_t g_cache_n = 0;
#define CACHE_MAX ((Py_ssize_t)1 << 22)   /* ids beyond this get a fresh object each */

static PyObject *id_object(int32_t v) {
    if (v < 0 || (Py_ssize_t)v >= CACHE_MAX) return PyLong_FromLong((long)v);
    if ((Py_ssize_t)v >= g_cache_n) {
        Py_ssize_t n = g_cache_n ? g_cache_n : 65536;
        while (n <= (Py_ssize_t)v) n *= 2;
        PyObject **c = (PyObject **)PyMem_Realloc(g_cache, (size_t)n * sizeof(PyObject *));
        if (!c) return PyErr_NoMemory();
        memset(c + g_cache_n, 0, (size_t)(n - g_cache_n) * sizeof(PyObject *));
        g_cache = c;
        g_cache_n = n;
    }
    PyObject *o = g_cache[v];
    if (!o) {
        o = PyLong_FromLong((long)v);
        if (!o) return NULL;
        g_cache[v] = o;
    }
    Py_INCREF(o);
    return o;
}

static int get_buf(PyObject *obj, Py_buffer *b, Py_ssize_t itemsize, const char *name) {
    if (PyObject_GetBuffer(obj, b, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) < 0) return -1;
    if (b->itemsize != itemsize) {
        PyErr_Format(PyExc_TypeError, "%s: expected %zd-byte items, got %zd", name, itemsize, b->itemsize);
        PyBuffer_Release(b);
        return -1;
    }
    return 0;
}

/* csr_lists(ids int32[], id_off uint64[n+1], status int32[n], none uint8[n] or None, ok, keep_failed)
 *   -> [(list of ids, status), ...]
 * String i: ([], ok) if none[i]; its ids if status[i] == ok or keep_failed; else ([], status[i]). */
static PyObject *csr_lists(PyObject *self, PyObject *args) {
    (void)self;
    PyObject *o_ids, *o_off, *o_st, *o_none;
    int ok, keep_failed;
    if (!PyArg_ParseTuple(args, "OOOOii", &o_ids, &o_off, &o_st, &o_none, &ok, &keep_failed)) return NULL;
    Py_buffer bi, bo, bs, bn;
    int have_none = o_none != Py_None;
    if (get_buf(o_ids, &bi, 4, "ids") < 0) return NULL;
    if (get_buf(o_off, &bo, 8, "id_off") < 0) { PyBuffer_Release(&bi); return NULL; }
    if (get_buf(o_st, &bs, 4, "status") < 0) { PyBuffer_Release(&bi); PyBuffer_Release(&bo); return NULL; }
    if (have_none && get_buf(o_none, &bn, 1, "none") < 0) {
        PyBuffer_Release(&bi); PyBuffer_Release(&bo); PyBuffer_Release(&bs);
        return NULL;
    }
    PyObject *out = NULL;
    const int32_t *ids = (const int32_t *)bi.buf;
    const uint64_t *off = (const uint64_t *)bo.buf;
    const int32_t *st = (const int32_t *)bs.buf;
    const uint8_t *none = have_none ? (const uint8_t *)bn.buf : NULL;
    const Py_ssize_t n_ids = bi.len / 4, n = bs.len / 4;
    if (bo.len / 8 < n + 1 || (have_none && bn.len < n)) {
        PyErr_SetString(PyExc_ValueError, "csr_lists: id_off needs n+1 entries (and none n)");
        goto done;
    }
    out = PyList_New(n);
    if (!out) goto done;
    for (Py_ssize_t i = 0; i < n; i++) {
        const int s = none && none[i] ? ok : st[i];
        const int take = (!none || !none[i]) && (s == ok || keep_failed);
        const uint64_t a = take ? off[i] - off[0] : 0, b = take ? off[i + 1] - off[0] : 0;
        if (b < a || (Py_ssize_t)b > n_ids) {
            PyErr_SetString(PyExc_ValueError, "csr_lists: offsets out of range");
            Py_CLEAR(out);
            goto done;
        }
        PyObject *lst = PyList_New((Py_ssize_t)(b - a));
        if (!lst) { Py_CLEAR(out); goto done; }
        for (uint64_t k = a; k < b; k++) {
            PyObject *v = id_object(ids[k]);
            if (!v) { Py_DECREF(lst); Py_CLEAR(out); goto done; }
            PyList_SET_ITEM(lst, (Py_ssize_t)(k - a), v);
        }
        PyObject *so = PyLong_FromLong(s);
        PyObject *tup = so ? PyTuple_Pack(2, lst, so) : NULL;
        Py_DECREF(lst);
        Py_XDECREF(so);
        if (!tup) { Py_CLEAR(out); goto done; }
        PyList_SET_ITEM(out, i, tup);
    }
done:
    PyBuffer_Release(&bi);
    PyBuffer_Release(&bo);
    PyBuffer_Release(&bs);
    if (have_none) PyBuffer_Release(&bn);
    return out;
}

static PyMethodDef methods[] = {
    {"csr_lists", csr_lists, METH_VARARGS, "CSR ids -> [(List[int], status)] per string"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_pylists", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__pylists(void) { return PyModule_Create(&module); }
