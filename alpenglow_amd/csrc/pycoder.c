/* CPython binding of the per-call coder entry points (ag_rs_coder_shred / _deshred) for
 * alpenglow_amd.rs.ReedSolomonCoder: the argument marshalling of the ctypes path (64 shred
 * pointers, lengths and data flags built as ctypes arrays, three zero-filled result buffers,
 * 64 slices) cost more than the device round trip it wraps (tools/bench_latency.py).  Here one
 * C loop reads the shred list, the results are written straight into bytes objects of their
 * final size, and the GIL is released around the device call.
 *
 * The library's entry points come in as addresses (bind(), from the ctypes handle of
 * libalpenglow_rs.so), so this module links nothing and follows the library rs.py loaded.
 * Host code only: no HIP call of its own. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

#include "alpenglow_rs.h"

typedef __typeof__(ag_rs_coder_shred)* shred_fn;
typedef __typeof__(ag_rs_coder_deshred)* deshred_fn;
typedef __typeof__(ag_rs_coder_num_coding)* num_coding_fn;

static shred_fn g_shred;
static deshred_fn g_deshred;
static num_coding_fn g_num_coding;

enum { kTotal = AG_RS_TOTAL_SHREDS, kData = AG_RS_DATA_SHREDS };

static PyObject* bind(PyObject* self, PyObject* args) {
  unsigned long long a, b, n;
  (void)self;
  if (!PyArg_ParseTuple(args, "KKK", &a, &b, &n)) return NULL;
  g_shred = (shred_fn)(uintptr_t)a;
  g_deshred = (deshred_fn)(uintptr_t)b;
  g_num_coding = (num_coding_fn)(uintptr_t)n;
  Py_RETURN_NONE;
}

/* The library writes num_coding * S coding bytes whatever the caller says: the caller's count
 * must be the coder's own, or the bytes object it sizes would overflow. */
static int check_num_coding(unsigned long long h, Py_ssize_t nc) {
  size_t own = 0;
  if (nc < 0) {
    PyErr_Format(PyExc_ValueError, "num_coding %zd < 0", nc);
    return -1;
  }
  if (g_num_coding((const ag_rs_coder*)(uintptr_t)h, &own) != 0) {
    PyErr_Format(PyExc_ValueError, "pycoder: not a coder handle");
    return -1;
  }
  if ((size_t)nc != own) {
    PyErr_Format(PyExc_ValueError, "num_coding %zd, the coder has %zu", nc, own);
    return -1;
  }
  return 0;
}

/* shred(coder, payload, num_coding) -> (status, data, coding, S): data / coding are the
 * 32 resp. num_coding shreds of S bytes, contiguous (reed_solomon.rs:88-128). */
static PyObject* shred(PyObject* self, PyObject* args) {
  unsigned long long h;
  Py_buffer pay;
  Py_ssize_t nc;
  (void)self;
  if (!g_shred) return PyErr_Format(PyExc_RuntimeError, "pycoder: bind() not called");
  if (!PyArg_ParseTuple(args, "Ky*n", &h, &pay, &nc)) return NULL;
  if (check_num_coding(h, nc) < 0) {
    PyBuffer_Release(&pay);
    return NULL;
  }
  /* padding 0x80 00.. to a multiple of 2 * DATA_SHREDS: S as the library computes it */
  const size_t len = (size_t)pay.len;
  const size_t S = (len + (2 * kData - len % (2 * kData))) / kData;
  PyObject* data = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)(kData * S));
  PyObject* coding = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)((size_t)nc * S));
  if (!data || !coding) {
    Py_XDECREF(data);
    Py_XDECREF(coding);
    PyBuffer_Release(&pay);
    return NULL;
  }
  size_t sb = 0;
  int st;
  Py_BEGIN_ALLOW_THREADS
  st = g_shred((ag_rs_coder*)(uintptr_t)h, (const uint8_t*)pay.buf, len, (uint8_t*)PyBytes_AS_STRING(data),
               (uint8_t*)PyBytes_AS_STRING(coding), &sb);
  Py_END_ALLOW_THREADS
  PyBuffer_Release(&pay);
  if (st == 0 && sb != S) {
    Py_DECREF(data);
    Py_DECREF(coding);
    return PyErr_Format(PyExc_RuntimeError, "pycoder: shred size %zu, expected %zu", sb, S);
  }
  return Py_BuildValue("(iNNn)", st, data, coding, (Py_ssize_t)sb);
}

/* deshred(coder, shreds, data_shreds, num_coding) -> (status, payload, data, coding, S):
 * shreds = TOTAL_SHREDS entries, each None or (is_data, bytes-like) (shredder.rs:282). */
static PyObject* deshred(PyObject* self, PyObject* args) {
  unsigned long long h;
  PyObject* seq;
  Py_ssize_t ds, nc;
  (void)self;
  if (!g_deshred) return PyErr_Format(PyExc_RuntimeError, "pycoder: bind() not called");
  if (!PyArg_ParseTuple(args, "KOnn", &h, &seq, &ds, &nc)) return NULL;
  PyObject* fast = PySequence_Fast(seq, "shreds must be a sequence");
  if (!fast) return NULL;
  if (PySequence_Fast_GET_SIZE(fast) != kTotal) {
    Py_DECREF(fast);
    return PyErr_Format(PyExc_ValueError, "expected %d shred slots", kTotal);
  }
  PyObject** items = PySequence_Fast_ITEMS(fast);
  Py_buffer views[kTotal];
  const uint8_t* ptrs[kTotal];
  size_t lens[kTotal];
  uint8_t isd[kTotal];
  int held[kTotal];
  size_t cap = 1;
  PyObject* result = NULL;
  int i;
  for (i = 0; i < kTotal; ++i) {
    held[i] = 0;
    ptrs[i] = NULL;
    lens[i] = 0;
    isd[i] = 0;
  }
  for (i = 0; i < kTotal; ++i) {
    PyObject* it = items[i];
    if (it == Py_None) continue;
    if (!PyTuple_Check(it) || PyTuple_GET_SIZE(it) != 2) {
      PyErr_Format(PyExc_TypeError, "shred %d: expected None or (is_data, bytes)", i);
      goto done;
    }
    const int flag = PyObject_IsTrue(PyTuple_GET_ITEM(it, 0));
    if (flag < 0 || PyObject_GetBuffer(PyTuple_GET_ITEM(it, 1), &views[i], PyBUF_SIMPLE) < 0) goto done;
    held[i] = 1;
    ptrs[i] = (const uint8_t*)views[i].buf;
    lens[i] = (size_t)views[i].len;
    isd[i] = (uint8_t)flag;
    if (lens[i] > cap) cap = lens[i];
  }
  if (check_num_coding(h, nc) < 0) goto done;
  {
    PyObject* payload = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)(kData * cap));
    PyObject* data = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)(kData * cap));
    PyObject* coding = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)((size_t)nc * cap));
    if (!payload || !data || !coding) {
      Py_XDECREF(payload);
      Py_XDECREF(data);
      Py_XDECREF(coding);
      goto done;
    }
    size_t plen = 0, sb = 0;
    int st;
    Py_BEGIN_ALLOW_THREADS
    st = g_deshred((ag_rs_coder*)(uintptr_t)h, (size_t)ds, ptrs, lens, isd, (uint8_t*)PyBytes_AS_STRING(payload),
                   &plen, (uint8_t*)PyBytes_AS_STRING(data), (uint8_t*)PyBytes_AS_STRING(coding), &sb);
    Py_END_ALLOW_THREADS
    if (st != 0) {
      plen = 0;
      sb = 0;
    }
    if (_PyBytes_Resize(&payload, (Py_ssize_t)plen) < 0 || _PyBytes_Resize(&data, (Py_ssize_t)(kData * sb)) < 0 ||
        _PyBytes_Resize(&coding, (Py_ssize_t)((size_t)nc * sb)) < 0) {
      Py_XDECREF(payload);
      Py_XDECREF(data);
      Py_XDECREF(coding);
      goto done;
    }
    result = Py_BuildValue("(iNNNn)", st, payload, data, coding, (Py_ssize_t)sb);
  }
done:
  for (i = 0; i < kTotal; ++i)
    if (held[i]) PyBuffer_Release(&views[i]);
  Py_DECREF(fast);
  return result;
}

static PyMethodDef methods[] = {
    {"bind", bind, METH_VARARGS, "bind(shred_addr, deshred_addr, num_coding_addr)"},
    {"shred", shred, METH_VARARGS, "shred(coder, payload, num_coding) -> (status, data, coding, S)"},
    {"deshred", deshred, METH_VARARGS, "deshred(coder, shreds, data_shreds, num_coding) -> (status, payload, data, coding, S)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_pycoder", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__pycoder(void) { return PyModule_Create(&module); }
