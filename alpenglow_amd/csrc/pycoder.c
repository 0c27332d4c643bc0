/* CPython binding of the per-call coder entry points (ag_rs_coder_shred / _deshred) for
 * alpenglow_amd.rs.ReedSolomonCoder, and of the crate-API encoder / decoder calls for
 * ReedSolomonEncoder / ReedSolomonDecoder: the argument marshalling of the ctypes path (64 shred
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
typedef __typeof__(ag_rs_encoder_add_original_shard)* enc_add_fn;
typedef __typeof__(ag_rs_encoder_encode)* enc_encode_fn;
typedef __typeof__(ag_rs_encoder_recovery)* enc_recovery_fn;
typedef __typeof__(ag_rs_decoder_add_original_shard)* dec_add_fn;
typedef __typeof__(ag_rs_decoder_decode)* dec_decode_fn;
typedef __typeof__(ag_rs_decoder_restored_original)* dec_restored_fn;

static shred_fn g_shred;
static deshred_fn g_deshred;
static num_coding_fn g_num_coding;
static enc_add_fn g_enc_add;
static enc_encode_fn g_enc_encode;
static enc_recovery_fn g_enc_recovery;
static dec_add_fn g_dec_add_o, g_dec_add_r;
static dec_decode_fn g_dec_decode;
static dec_restored_fn g_dec_restored;

enum { kTotal = AG_RS_TOTAL_SHREDS, kData = AG_RS_DATA_SHREDS };

/* bind(shred, deshred, num_coding, encoder add / encode / recovery, decoder add original /
 * add recovery / decode / restored_original): the library's entry points by address */
static PyObject* bind(PyObject* self, PyObject* args) {
  unsigned long long a[10];
  (void)self;
  if (!PyArg_ParseTuple(args, "KKKKKKKKKK", &a[0], &a[1], &a[2], &a[3], &a[4], &a[5], &a[6], &a[7], &a[8], &a[9]))
    return NULL;
  g_shred = (shred_fn)(uintptr_t)a[0];
  g_deshred = (deshred_fn)(uintptr_t)a[1];
  g_num_coding = (num_coding_fn)(uintptr_t)a[2];
  g_enc_add = (enc_add_fn)(uintptr_t)a[3];
  g_enc_encode = (enc_encode_fn)(uintptr_t)a[4];
  g_enc_recovery = (enc_recovery_fn)(uintptr_t)a[5];
  g_dec_add_o = (dec_add_fn)(uintptr_t)a[6];
  g_dec_add_r = (dec_add_fn)(uintptr_t)a[7];
  g_dec_decode = (dec_decode_fn)(uintptr_t)a[8];
  g_dec_restored = (dec_restored_fn)(uintptr_t)a[9];
  Py_RETURN_NONE;
}

/* ReedSolomonEncoder / ReedSolomonDecoder (INTEGRATION.md Route A) without ctypes marshalling:
 * each crate call is one C call here, and the results come back as bytes objects in one loop.
 * Every function returns the library status (0 = OK) or raises on malformed arguments. */
static PyObject* enc_add(PyObject* self, PyObject* args) {
  unsigned long long h;
  Py_buffer b;
  (void)self;
  if (!g_enc_add) return PyErr_Format(PyExc_RuntimeError, "pycoder: bind() not called");
  if (!PyArg_ParseTuple(args, "Ky*", &h, &b)) return NULL;
  const int st = g_enc_add((ag_rs_encoder*)(uintptr_t)h, (const uint8_t*)b.buf, (size_t)b.len);
  PyBuffer_Release(&b);
  return PyLong_FromLong(st);
}

/* enc_encode(encoder, recovery_count) -> (status, [recovery shards]) */
static PyObject* enc_encode(PyObject* self, PyObject* args) {
  unsigned long long h;
  Py_ssize_t m, j;
  int st;
  (void)self;
  if (!g_enc_encode) return PyErr_Format(PyExc_RuntimeError, "pycoder: bind() not called");
  if (!PyArg_ParseTuple(args, "Kn", &h, &m)) return NULL;
  if (m < 0) return PyErr_Format(PyExc_ValueError, "recovery_count %zd < 0", m);
  ag_rs_encoder* e = (ag_rs_encoder*)(uintptr_t)h;
  Py_BEGIN_ALLOW_THREADS
  st = g_enc_encode(e);
  Py_END_ALLOW_THREADS
  PyObject* out = PyList_New(0);
  if (!out) return NULL;
  for (j = 0; st == 0 && j < m; ++j) {
    const uint8_t* p = NULL;
    size_t len = 0;
    if ((st = g_enc_recovery(e, (size_t)j, &p, &len)) != 0) break;
    PyObject* b = PyBytes_FromStringAndSize((const char*)p, (Py_ssize_t)len);
    if (!b || PyList_Append(out, b) < 0) {
      Py_XDECREF(b);
      Py_DECREF(out);
      return NULL;
    }
    Py_DECREF(b);
  }
  return Py_BuildValue("(iN)", st, out);
}

/* dec_add(decoder, is_original, index, shard) -> status */
static PyObject* dec_add(PyObject* self, PyObject* args) {
  unsigned long long h;
  int orig;
  Py_ssize_t idx;
  Py_buffer b;
  (void)self;
  if (!g_dec_add_o) return PyErr_Format(PyExc_RuntimeError, "pycoder: bind() not called");
  if (!PyArg_ParseTuple(args, "Kpny*", &h, &orig, &idx, &b)) return NULL;
  if (idx < 0) {
    PyBuffer_Release(&b);
    return PyErr_Format(PyExc_ValueError, "index %zd < 0", idx);
  }
  const int st = (orig ? g_dec_add_o : g_dec_add_r)((ag_rs_decoder*)(uintptr_t)h, (size_t)idx,
                                                    (const uint8_t*)b.buf, (size_t)b.len);
  PyBuffer_Release(&b);
  return PyLong_FromLong(st);
}

/* dec_decode(decoder, original_count) -> (status, {index: restored original}) */
static PyObject* dec_decode(PyObject* self, PyObject* args) {
  unsigned long long h;
  Py_ssize_t k, i;
  int st;
  (void)self;
  if (!g_dec_decode) return PyErr_Format(PyExc_RuntimeError, "pycoder: bind() not called");
  if (!PyArg_ParseTuple(args, "Kn", &h, &k)) return NULL;
  if (k < 0) return PyErr_Format(PyExc_ValueError, "original_count %zd < 0", k);
  ag_rs_decoder* d = (ag_rs_decoder*)(uintptr_t)h;
  Py_BEGIN_ALLOW_THREADS
  st = g_dec_decode(d);
  Py_END_ALLOW_THREADS
  PyObject* out = PyDict_New();
  if (!out) return NULL;
  for (i = 0; st == 0 && i < k; ++i) {
    const uint8_t* p = NULL;
    size_t len = 0;
    if (g_dec_restored(d, (size_t)i, &p, &len) != 0) continue;  /* not restored (crate: None) */
    PyObject* key = PyLong_FromSsize_t(i);
    PyObject* b = PyBytes_FromStringAndSize((const char*)p, (Py_ssize_t)len);
    if (!key || !b || PyDict_SetItem(out, key, b) < 0) {
      Py_XDECREF(key);
      Py_XDECREF(b);
      Py_DECREF(out);
      return NULL;
    }
    Py_DECREF(key);
    Py_DECREF(b);
  }
  return Py_BuildValue("(iN)", st, out);
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
    {"bind", bind, METH_VARARGS, "bind(shred, deshred, num_coding, enc_add, enc_encode, enc_recovery, dec_add_o, "
                                 "dec_add_r, dec_decode, dec_restored)"},
    {"enc_add", enc_add, METH_VARARGS, "enc_add(encoder, shard) -> status"},
    {"enc_encode", enc_encode, METH_VARARGS, "enc_encode(encoder, recovery_count) -> (status, [recovery])"},
    {"dec_add", dec_add, METH_VARARGS, "dec_add(decoder, is_original, index, shard) -> status"},
    {"dec_decode", dec_decode, METH_VARARGS, "dec_decode(decoder, original_count) -> (status, {i: restored})"},
    {"shred", shred, METH_VARARGS, "shred(coder, payload, num_coding) -> (status, data, coding, S)"},
    {"deshred", deshred, METH_VARARGS, "deshred(coder, shreds, data_shreds, num_coding) -> (status, payload, data, coding, S)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_pycoder", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__pycoder(void) { return PyModule_Create(&module); }
