/* host_ext.c -- _coup_host: the CPython binding of libcoup_mi355x.so's
 * host-resident State ops (coup_host_state_*, csrc/coup_host.cpp), for the
 * per-game pyspiel facade.  The same C functions are reachable through
 * ctypes; this module only removes ctypes' per-call cost (~0.7 us of a
 * ~1.7 us apply_action from Python), the part that dominates a one-op-per-
 * node walk (outcome_sampling_mccfr.py:81-87).  It links the HIP library:
 * there is no build of it without libcoup_mi355x.so.
 *
 *   bind(result_type)               -> None: init / apply return result_type instances from now on
 *   init()                          -> (raw, legal_mask, cur_player, terminal, ok, unrepresentable),
 *                                      or after bind a result_type with those keys and ._raw
 *   apply(raw, action, flags)       -> the same for the state after State::ApplyAction
 *   step(raw, action, mode, seed, env_id) -> the same for rl_environment's reset / step (raw may be None
 *                                      with mode COUP_SLOT_INIT)
 *   string(raw, kind, player)       -> str (0 ObservationString, 1 InformationStateString, 2 ToString)
 *   tensors(raw, obs, info)         -> None (float32 [2][98] / [2][2492] into obs / info, None = skip)
 *   float_lists(rows_f32, rows, cols) -> rows lists of floats (the time steps' tensors)
 *
 * obs, info and rows_f32 are C-contiguous float32 buffers (numpy arrays:
 * the buffer protocol, no ctypes address lookup per call) or integer
 * addresses (0 = skip). *
 * raw is the state's 128-byte coup_slot_result (bytes). */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <math.h>
#include <string.h>

#include "coup_mi355x.h"

/* bind(result_type): the facade's result class (a dict subclass with a
 * `_raw` slot, pyspiel._Result); init / apply then return instances of it
 * directly, keys filled here, instead of a tuple the caller repacks. */
static PyObject* g_result_type = NULL;
static PyObject *k_legal, *k_player, *k_terminal, *k_ok, *k_unrep, *k_raw;

static PyObject* result_tuple(const coup_slot_result* r) {
  PyObject* raw = PyBytes_FromStringAndSize((const char*)r, (Py_ssize_t)sizeof(*r));
  if (!raw) return NULL;
  if (!g_result_type)
    return Py_BuildValue("(NIiOOO)", raw, (unsigned int)r->legal_mask, (int)r->cur_player,
                         r->terminal ? Py_True : Py_False, r->ok ? Py_True : Py_False,
                         r->unrepresentable ? Py_True : Py_False);
  PyObject* q = PyObject_CallNoArgs(g_result_type);
  if (!q) {
    Py_DECREF(raw);
    return NULL;
  }
  PyObject* lm = PyLong_FromUnsignedLong(r->legal_mask);
  PyObject* cp = PyLong_FromLong(r->cur_player);
  int bad = !lm || !cp || PyDict_SetItem(q, k_legal, lm) || PyDict_SetItem(q, k_player, cp) ||
            PyDict_SetItem(q, k_terminal, r->terminal ? Py_True : Py_False) ||
            PyDict_SetItem(q, k_ok, r->ok ? Py_True : Py_False) ||
            PyDict_SetItem(q, k_unrep, r->unrepresentable ? Py_True : Py_False) || PyObject_SetAttr(q, k_raw, raw);
  Py_XDECREF(lm);
  Py_XDECREF(cp);
  Py_DECREF(raw);
  if (bad) {
    Py_DECREF(q);
    return NULL;
  }
  return q;
}

static PyObject* py_bind(PyObject* self, PyObject* type) {
  (void)self;
  if (!PyType_Check(type) || !PyType_IsSubtype((PyTypeObject*)type, &PyDict_Type)) {
    PyErr_SetString(PyExc_TypeError, "bind(result_type): a dict subclass");
    return NULL;
  }
  if (!k_legal) {
    k_legal = PyUnicode_InternFromString("legal_mask");
    k_player = PyUnicode_InternFromString("current_player");
    k_terminal = PyUnicode_InternFromString("terminal");
    k_ok = PyUnicode_InternFromString("ok");
    k_unrep = PyUnicode_InternFromString("unrepresentable");
    k_raw = PyUnicode_InternFromString("_raw");
    if (!k_legal || !k_player || !k_terminal || !k_ok || !k_unrep || !k_raw) return NULL;
  }
  Py_INCREF(type);
  Py_XSETREF(g_result_type, type);
  Py_RETURN_NONE;
}

static int as_state(PyObject* o, const coup_slot_result** st) {
  if (!PyBytes_Check(o) || PyBytes_GET_SIZE(o) != (Py_ssize_t)sizeof(coup_slot_result)) {
    PyErr_SetString(PyExc_ValueError, "a host state is 128 bytes (coup_slot_result)");
    return 0;
  }
  *st = (const coup_slot_result*)PyBytes_AS_STRING(o);
  return 1;
}

static PyObject* py_init(PyObject* self, PyObject* args) {
  (void)self;
  (void)args;
  coup_slot_result r;
  if (coup_host_state_init(&r) != COUP_OK) {
    PyErr_SetString(PyExc_RuntimeError, "coup_host_state_init failed");
    return NULL;
  }
  return result_tuple(&r);
}

static PyObject* py_apply(PyObject* self, PyObject* const* args, Py_ssize_t n) {
  (void)self;
  if (n != 3) {
    PyErr_SetString(PyExc_TypeError, "apply(raw, action, flags)");
    return NULL;
  }
  const coup_slot_result* st;
  if (!as_state(args[0], &st)) return NULL;
  const long action = PyLong_AsLong(args[1]), flags = PyLong_AsLong(args[2]);
  if (PyErr_Occurred()) return NULL;
  coup_slot_result r;
  if (action < 0 || action > 127 || coup_host_state_apply(st, (int)action, (int)flags, &r) != COUP_OK) {
    PyErr_Format(PyExc_ValueError, "coup_host_state_apply: invalid action %ld", action);
    return NULL;
  }
  return result_tuple(&r);
}

static PyObject* py_step(PyObject* self, PyObject* const* args, Py_ssize_t n) {
  (void)self;
  if (n != 5) {
    PyErr_SetString(PyExc_TypeError, "step(raw_or_None, action, mode, seed, env_id)");
    return NULL;
  }
  const coup_slot_result* st = NULL;
  if (args[0] != Py_None && !as_state(args[0], &st)) return NULL;
  const long action = PyLong_AsLong(args[1]), mode = PyLong_AsLong(args[2]);
  const unsigned long long seed = PyLong_AsUnsignedLongLongMask(args[3]);
  const unsigned long env_id = PyLong_AsUnsignedLong(args[4]);
  if (PyErr_Occurred()) return NULL;
  coup_slot_result r;
  if (action < -1 || action > 127 ||
      coup_host_state_step(st, (int)action, (int)mode, (uint64_t)seed, (uint32_t)env_id, &r) != COUP_OK) {
    PyErr_Format(PyExc_ValueError, "coup_host_state_step: action %ld mode %ld", action, mode);
    return NULL;
  }
  return result_tuple(&r);
}

static PyObject* py_string(PyObject* self, PyObject* const* args, Py_ssize_t n) {
  (void)self;
  if (n != 3) {
    PyErr_SetString(PyExc_TypeError, "string(raw, kind, player)");
    return NULL;
  }
  const coup_slot_result* st;
  if (!as_state(args[0], &st)) return NULL;
  const long kind = PyLong_AsLong(args[1]), player = PyLong_AsLong(args[2]);
  if (PyErr_Occurred()) return NULL;
  char buf[1024];
  const int64_t len = coup_host_state_string(st, (int)kind, (int)player, buf, (int64_t)sizeof(buf));
  if (len < 0) {
    PyErr_Format(PyExc_ValueError, "coup_host_state_string: kind %ld player %ld", kind, player);
    return NULL;
  }
  if (len < (int64_t)sizeof(buf)) return PyUnicode_DecodeASCII(buf, (Py_ssize_t)len, NULL);
  char* big = (char*)PyMem_Malloc((size_t)len + 1);
  if (!big) return PyErr_NoMemory();
  coup_host_state_string(st, (int)kind, (int)player, big, len + 1);
  PyObject* s = PyUnicode_DecodeASCII(big, (Py_ssize_t)len, NULL);
  PyMem_Free(big);
  return s;
}

/* A float32 buffer argument: None or an integer address (0 = none), or a
 * C-contiguous buffer of at least `floats` elements (released by
 * release_floats). */
static int get_floats(PyObject* o, Py_ssize_t floats, int writable, Py_buffer* view, float** out) {
  view->obj = NULL;
  *out = NULL;
  if (o == Py_None) return 1;
  if (PyLong_Check(o)) {
    *out = (float*)PyLong_AsVoidPtr(o);
    return !PyErr_Occurred();
  }
  if (PyObject_GetBuffer(o, view, (writable ? PyBUF_WRITABLE : 0) | PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0)
    return 0;
  if (view->itemsize != 4 || (view->format && strcmp(view->format, "f") != 0) || view->len < floats * 4) {
    PyBuffer_Release(view);
    view->obj = NULL;
    PyErr_SetString(PyExc_ValueError, "expected a C-contiguous float32 buffer of the tensor's size");
    return 0;
  }
  *out = (float*)view->buf;
  return 1;
}

static void release_floats(Py_buffer* view) {
  if (view->obj) PyBuffer_Release(view);
}

static PyObject* py_tensors(PyObject* self, PyObject* const* args, Py_ssize_t n) {
  (void)self;
  if (n != 3) {
    PyErr_SetString(PyExc_TypeError, "tensors(raw, obs, info)");
    return NULL;
  }
  const coup_slot_result* st;
  if (!as_state(args[0], &st)) return NULL;
  Py_buffer vo, vi;
  float *obs, *info;
  if (!get_floats(args[1], 2 * COUP_OBS_SIZE, 1, &vo, &obs)) return NULL;
  if (!get_floats(args[2], 2 * COUP_INFO_STATE_SIZE, 1, &vi, &info)) {
    release_floats(&vo);
    return NULL;
  }
  const int rc = coup_host_state_tensors(st, obs, info);
  release_floats(&vo);
  release_floats(&vi);
  if (rc != COUP_OK) {
    PyErr_SetString(PyExc_RuntimeError, "coup_host_state_tensors failed");
    return NULL;
  }
  Py_RETURN_NONE;
}

/* float_lists(addr, rows, cols): rows x cols contiguous float32 at addr as a
 * list of `rows` Python lists of floats -- the time steps' tensors
 * (rl_environment.py:243-248 hands them out as lists).  Integral values
 * 0..15 (every element of both tensors: one-hots, coin counts) share a few
 * float objects each, so building and later copying / collecting the lists
 * touches a few objects instead of 2 x 2492 fresh ones per env and step;
 * any other value gets its own float, exactly float(x) of the float32.
 * Column c takes copy c % kCopies of its value: the reference-count updates
 * of one list (when built, and again when freed) then form kCopies
 * independent chains instead of one store-to-load chain through a single
 * object's count, ~4x faster for an info-state row. */
enum { kCopies = 8 };
static PyObject* g_small[16][kCopies];

static PyObject* build_lists(const float* src, Py_ssize_t rows, Py_ssize_t cols, int untrack);

/* float_lists(rows_f32, rows, cols[, untrack = 1]).  untrack = 0 keeps the
 * rows in the cyclic collector (the pyspiel State tensor accessors: one row,
 * an ordinary list a caller may grow into a cycle); 1 leaves them out of it
 * (rl_environment time steps: the facade's documented contract, see
 * build_lists). */
static PyObject* py_float_lists(PyObject* self, PyObject* const* args, Py_ssize_t n) {
  (void)self;
  if (n != 3 && n != 4) {
    PyErr_SetString(PyExc_TypeError, "float_lists(rows_f32, rows, cols[, untrack])");
    return NULL;
  }
  const Py_ssize_t rows = PyLong_AsSsize_t(args[1]), cols = PyLong_AsSsize_t(args[2]);
  const long untrack = n == 4 ? PyLong_AsLong(args[3]) : 1;
  if (PyErr_Occurred()) return NULL;
  if (rows < 0 || cols < 0) {
    PyErr_SetString(PyExc_ValueError, "float_lists: bad shape");
    return NULL;
  }
  Py_buffer view;
  float* buf;
  if (!get_floats(args[0], rows * cols, 0, &view, &buf)) return NULL;
  PyObject* res = build_lists(buf, rows, cols, untrack != 0);
  release_floats(&view);
  return res;
}

/* A new reference for a non-zero element of column copy j. */
static PyObject* element(float v, int j) {
  const int k = (v >= 0.0f && v < 16.0f) ? (int)v : -1; /* converted only where it fits */
  if (k >= 0 && (float)k == v && !(v == 0.0f && signbit(v))) {
    Py_INCREF(g_small[k][j]);
    return g_small[k][j];
  }
  return PyFloat_FromDouble((double)v);
}

static PyObject* build_lists(const float* src, Py_ssize_t rows, Py_ssize_t cols, int untrack) {
  if (!src) {
    PyErr_SetString(PyExc_ValueError, "float_lists: bad buffer");
    return NULL;
  }
  if (!g_small[15][kCopies - 1]) /* filled in order, the last one only when all succeeded */
    for (int k = 0; k < 16; ++k)
      for (int j = 0; j < kCopies; ++j)
        if (!g_small[k][j] && !(g_small[k][j] = PyFloat_FromDouble((double)k))) return NULL;
  PyObject* out = PyList_New(rows);
  if (!out) return NULL;
  for (Py_ssize_t r = 0; r < rows; ++r) {
    PyObject* row = PyList_New(cols);
    if (!row) {
      Py_DECREF(out);
      return NULL;
    }
    const float* x = src + r * cols;
    /* +0.0 (most elements) is stored without touching its object: the
     * references are counted per copy in registers and added once */
    Py_ssize_t zc[kCopies] = {0};
    int failed = 0;
    Py_ssize_t c = 0;
#define COUP_ONE(J)                                  \
  {                                                  \
    const float v = x[c + (J)];                      \
    uint32_t u;                                      \
    memcpy(&u, &v, sizeof u);                        \
    PyObject* o;                                     \
    if (u == 0u) {                                   \
      o = g_small[0][(J)];                           \
      ++zc[(J)];                                     \
    } else if (!(o = element(v, (J)))) {             \
      failed = 1;                                    \
      break;                                         \
    }                                                \
    PyList_SET_ITEM(row, c + (J), o);                \
  }
    for (; c + kCopies <= cols; c += kCopies) {
      do {
        COUP_ONE(0) COUP_ONE(1) COUP_ONE(2) COUP_ONE(3) COUP_ONE(4) COUP_ONE(5) COUP_ONE(6) COUP_ONE(7)
      } while (0);
      if (failed) break;
    }
    for (; !failed && c < cols; ++c) {
      const float v = x[c];
      uint32_t u;
      memcpy(&u, &v, sizeof u);
      PyObject* o;
      if (u == 0u) {
        o = g_small[0][c % kCopies];
        ++zc[c % kCopies];
      } else if (!(o = element(v, (int)(c % kCopies)))) {
        failed = 1;
        break;
      }
      PyList_SET_ITEM(row, c, o);
    }
#undef COUP_ONE
#ifndef Py_GIL_DISABLED
    /* under the GIL the counts are plain integers: add each copy's at once */
    for (int j = 0; j < kCopies; ++j) Py_SET_REFCNT(g_small[0][j], Py_REFCNT(g_small[0][j]) + zc[j]);
#else
    /* free-threaded builds split reference counts: one Py_INCREF per item */
    for (int j = 0; j < kCopies; ++j)
      for (Py_ssize_t q = 0; q < zc[j]; ++q) Py_INCREF(g_small[0][j]);
#endif
    if (failed) { /* the items set so far hold their references; the rest are NULL */
      Py_DECREF(row);
      Py_DECREF(out);
      return NULL;
    }
    /* a list of floats cannot be part of a reference cycle: keep it out of
     * the cyclic collector, which would otherwise visit its 2492 items in
     * every collection it survives (a 256-env vector step keeps ~500 such
     * lists alive across collections: +60% per env step, measured).  As
     * CPython does for tuples and dicts of atomic values; a caller that later
     * puts a container into such a list and builds a cycle through it only
     * leaves that cycle to be freed by hand (documented on
     * rl_environment.Environment; the State accessors pass untrack = 0). */
    if (untrack) PyObject_GC_UnTrack(row);
    PyList_SET_ITEM(out, r, row);
  }
  return out;
}

static PyMethodDef kMethods[] = {
    {"float_lists", (PyCFunction)(void (*)(void))py_float_lists, METH_FASTCALL, "float32 rows as lists of floats"},
    {"bind", py_bind, METH_O, "the result class init / apply return"},
    {"init", py_init, METH_NOARGS, "NewInitialState as a host state tuple"},
    {"step", (PyCFunction)(void (*)(void))py_step, METH_FASTCALL, "rl_environment's reset / step on a host state"},
    {"apply", (PyCFunction)(void (*)(void))py_apply, METH_FASTCALL, "State::ApplyAction on a host state"},
    {"string", (PyCFunction)(void (*)(void))py_string, METH_FASTCALL, "Observation / InformationState / ToString"},
    {"tensors", (PyCFunction)(void (*)(void))py_tensors, METH_FASTCALL, "both players' tensors into buffers"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_coup_host", NULL, -1, kMethods,
                                     NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__coup_host(void) { return PyModule_Create(&kModule); }
