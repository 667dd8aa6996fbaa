// Low-overhead CPython entry points for the host plane's hot calls.
//
// The mpi4py-compatible layer (mpi.py) calls these for plain C-contiguous
// buffers (NumPy arrays, bytearrays, CPU tensors' arrays): METH_FASTCALL
// functions that take the communicator as a raw pointer, borrow the buffer
// through the buffer protocol and infer the element type from its format
// string.  Per call this is ~0.1-0.2 us of Python-side work instead of the
// ~2.5 us of generic pybind11 dispatch + buffer-spec parsing, which is what a
// 100-element Send/Recv costs end to end (reference workload: mpi-test.py's
// 100 x int64 myAllreduce / p x int64 myAlltoall loops).
//
// Anything that is not a plain contiguous buffer makes the function return
// NotImplemented (no exception), and mpi.py falls back to its general path.
//
// Requests are kept in a handle table (an int per request instead of a
// pybind11 object); fwait() completes and frees a handle.
#include <Python.h>

#include <stdexcept>
#include <vector>

#include "shm_comm.hpp"

namespace ccmpi {

namespace {

struct View {
  Py_buffer v;
  bool ok = false;
  ~View() {
    if (ok) PyBuffer_Release(&v);
  }
  char* ptr() const { return static_cast<char*>(v.buf); }
  size_t nbytes() const { return (size_t)v.len; }
};

// 1 = got a C-contiguous view; 0 = not a plain buffer (no error set)
int view_of(PyObject* o, bool writable, bool fmt, View& out) {
  int flags = PyBUF_C_CONTIGUOUS | (writable ? PyBUF_WRITABLE : 0) | (fmt ? PyBUF_FORMAT : 0);
  if (PyObject_GetBuffer(o, &out.v, flags) != 0) {
    PyErr_Clear();
    return 0;
  }
  out.ok = true;
  return 1;
}

// element type from a struct-module format string; -1 if unknown
int dtype_of(const View& b) {
  const char* f = b.v.format ? b.v.format : "B";
  if (*f == '=' || *f == '<' || *f == '@') ++f;
  if (!f[0] || f[1]) return -1;
  const Py_ssize_t is = b.v.itemsize;
  switch (f[0]) {
    case 'b': return DT_I8;
    case 'B': return DT_U8;
    case 'h': return DT_I16;
    case 'H': return DT_U16;
    case 'i': return is == 4 ? DT_I32 : -1;
    case 'I': return is == 4 ? DT_U32 : -1;
    case 'l': return is == 8 ? DT_I64 : (is == 4 ? DT_I32 : -1);
    case 'L': return is == 8 ? DT_U64 : (is == 4 ? DT_U32 : -1);
    case 'q': return DT_I64;
    case 'Q': return DT_U64;
    case 'e': return DT_F16;
    case 'f': return DT_F32;
    case 'd': return DT_F64;
    case '?': return DT_BOOL;
    default: return -1;
  }
}

ShmComm* comm_of(PyObject* o) { return static_cast<ShmComm*>(PyLong_AsVoidPtr(o)); }

PyObject* not_impl() { Py_RETURN_NOTIMPLEMENTED; }

PyObject* status_tuple(const RequestPtr& r) {
  return Py_BuildValue("(iin)", r->st_source, r->st_tag, (Py_ssize_t)r->st_count);
}

// run `fn` with the GIL released, translating C++ exceptions
template <class F>
bool guarded(F&& fn) {
  std::string err;
  int kind = 0;
  Py_BEGIN_ALLOW_THREADS
  try {
    fn();
  } catch (const std::invalid_argument& e) {
    err = e.what();
    kind = 1;
  } catch (const std::exception& e) {
    err = e.what();
    kind = 2;
  }
  Py_END_ALLOW_THREADS
  if (kind) {
    PyErr_SetString(kind == 1 ? PyExc_ValueError : PyExc_RuntimeError, err.c_str());
    return false;
  }
  return true;
}

// same, but without releasing the GIL (calls that never block)
template <class F>
bool guarded_nb(F&& fn) {
  try {
    fn();
  } catch (const std::invalid_argument& e) {
    PyErr_SetString(PyExc_ValueError, e.what());
    return false;
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return false;
  }
  return true;
}

bool nargs_is(Py_ssize_t n, Py_ssize_t want, const char* name) {
  if (n == want) return true;
  PyErr_Format(PyExc_TypeError, "%s expects %zd arguments", name, want);
  return false;
}

// ---- request handles ------------------------------------------------------
struct Slot {
  ShmComm* comm = nullptr;
  RequestPtr req;
};
std::vector<Slot> g_slots;
std::vector<Py_ssize_t> g_free;

Py_ssize_t put(ShmComm* c, RequestPtr r) {
  Py_ssize_t h;
  if (!g_free.empty()) {
    h = g_free.back();
    g_free.pop_back();
  } else {
    h = (Py_ssize_t)g_slots.size();
    g_slots.emplace_back();
  }
  g_slots[h].comm = c;
  g_slots[h].req = std::move(r);
  return h;
}

Slot* slot_of(PyObject* o) {
  Py_ssize_t h = PyLong_AsSsize_t(o);
  if (h < 0 || h >= (Py_ssize_t)g_slots.size() || !g_slots[h].req) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "ccmpi: invalid request handle");
    return nullptr;
  }
  return &g_slots[h];
}

void release(PyObject* o) {
  Py_ssize_t h = PyLong_AsSsize_t(o);
  g_slots[h].req.reset();
  g_slots[h].comm = nullptr;
  g_free.push_back(h);
}

// ---- point to point -------------------------------------------------------
PyObject* f_send(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 4, "fsend")) return nullptr;
  View b;
  if (!view_of(a[1], false, false, b)) return not_impl();
  ShmComm* c = comm_of(a[0]);
  if (!c) return PyErr_Occurred() ? nullptr : (PyErr_SetString(PyExc_ValueError, "ccmpi: communicator freed"), nullptr);
  int dest = (int)PyLong_AsLong(a[2]), tag = (int)PyLong_AsLong(a[3]);
  if (PyErr_Occurred()) return nullptr;
  RequestPtr r;
  if (!guarded_nb([&] { r = c->isend(b.ptr(), b.nbytes(), dest, tag); })) return nullptr;
  if (!r->complete && !guarded([&] { c->wait(r); })) return nullptr;
  Py_RETURN_NONE;
}

PyObject* f_recv(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 4, "frecv")) return nullptr;
  View b;
  if (!view_of(a[1], true, false, b)) return not_impl();
  ShmComm* c = comm_of(a[0]);
  if (!c) return PyErr_Occurred() ? nullptr : (PyErr_SetString(PyExc_ValueError, "ccmpi: communicator freed"), nullptr);
  int src = (int)PyLong_AsLong(a[2]), tag = (int)PyLong_AsLong(a[3]);
  if (PyErr_Occurred()) return nullptr;
  RequestPtr r;
  if (!guarded_nb([&] { r = c->irecv(b.ptr(), b.nbytes(), src, tag); })) return nullptr;
  if (!guarded([&] { c->wait(r); })) return nullptr;
  return status_tuple(r);
}

PyObject* f_isend(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 4, "fisend")) return nullptr;
  View b;
  if (!view_of(a[1], false, false, b)) return not_impl();
  ShmComm* c = comm_of(a[0]);
  if (!c) return PyErr_Occurred() ? nullptr : (PyErr_SetString(PyExc_ValueError, "ccmpi: communicator freed"), nullptr);
  int dest = (int)PyLong_AsLong(a[2]), tag = (int)PyLong_AsLong(a[3]);
  if (PyErr_Occurred()) return nullptr;
  RequestPtr r;
  if (!guarded_nb([&] { r = c->isend(b.ptr(), b.nbytes(), dest, tag); })) return nullptr;
  return PyLong_FromSsize_t(put(c, std::move(r)));
}

PyObject* f_irecv(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 4, "firecv")) return nullptr;
  View b;
  if (!view_of(a[1], true, false, b)) return not_impl();
  ShmComm* c = comm_of(a[0]);
  if (!c) return PyErr_Occurred() ? nullptr : (PyErr_SetString(PyExc_ValueError, "ccmpi: communicator freed"), nullptr);
  int src = (int)PyLong_AsLong(a[2]), tag = (int)PyLong_AsLong(a[3]);
  if (PyErr_Occurred()) return nullptr;
  RequestPtr r;
  if (!guarded_nb([&] { r = c->irecv(b.ptr(), b.nbytes(), src, tag); })) return nullptr;
  return PyLong_FromSsize_t(put(c, std::move(r)));
}

// fwait(handle) -> (source, tag, bytes); frees the handle
PyObject* f_wait(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 1, "fwait")) return nullptr;
  Slot* s = slot_of(a[0]);
  if (!s) return nullptr;
  RequestPtr r = s->req;
  ShmComm* c = s->comm;
  release(a[0]);
  if (!r->complete && !guarded([&] { c->wait(r); })) return nullptr;
  if (r->truncated) {
    PyErr_SetString(PyExc_RuntimeError, "ccmpi: message truncated (receive buffer too small)");
    return nullptr;
  }
  return status_tuple(r);
}

// ftest(handle) -> bool (the handle stays valid)
PyObject* f_test(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 1, "ftest")) return nullptr;
  Slot* s = slot_of(a[0]);
  if (!s) return nullptr;
  bool done = false;
  if (!guarded_nb([&] { done = s->comm->test(s->req); })) return nullptr;
  return PyBool_FromLong(done);
}

// fwaitall(list of handles): completes every request (handles stay valid)
PyObject* f_waitall(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 1, "fwaitall")) return nullptr;
  PyObject* seq = PySequence_Fast(a[0], "fwaitall expects a sequence of handles");
  if (!seq) return nullptr;
  Py_ssize_t m = PySequence_Fast_GET_SIZE(seq);
  std::vector<std::pair<ShmComm*, RequestPtr>> rs;
  rs.reserve(m);
  for (Py_ssize_t i = 0; i < m; ++i) {
    Slot* s = slot_of(PySequence_Fast_GET_ITEM(seq, i));
    if (!s) {
      Py_DECREF(seq);
      return nullptr;
    }
    if (!s->req->complete) rs.emplace_back(s->comm, s->req);
  }
  Py_DECREF(seq);
  if (!rs.empty() && !guarded([&] {
        for (auto& [c, r] : rs) c->wait(r);
      }))
    return nullptr;
  Py_RETURN_NONE;
}

PyObject* f_sendrecv(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 7, "fsendrecv")) return nullptr;
  View s, r;
  if (!view_of(a[1], false, false, s) || !view_of(a[4], true, false, r)) return not_impl();
  ShmComm* c = comm_of(a[0]);
  if (!c) return PyErr_Occurred() ? nullptr : (PyErr_SetString(PyExc_ValueError, "ccmpi: communicator freed"), nullptr);
  int dest = (int)PyLong_AsLong(a[2]), stag = (int)PyLong_AsLong(a[3]);
  int src = (int)PyLong_AsLong(a[5]), rtag = (int)PyLong_AsLong(a[6]);
  if (PyErr_Occurred()) return nullptr;
  RequestPtr rr;
  if (!guarded([&] { rr = c->sendrecv(s.ptr(), s.nbytes(), dest, stag, r.ptr(), r.nbytes(), src, rtag); }))
    return nullptr;
  return status_tuple(rr);
}

// ---- collectives ----------------------------------------------------------
PyObject* f_barrier(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 1, "fbarrier")) return nullptr;
  ShmComm* c = comm_of(a[0]);
  if (!c) return PyErr_Occurred() ? nullptr : (PyErr_SetString(PyExc_ValueError, "ccmpi: communicator freed"), nullptr);
  if (!guarded([&] { c->barrier(); })) return nullptr;
  Py_RETURN_NONE;
}

PyObject* f_bcast(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 3, "fbcast")) return nullptr;
  View b;
  if (!view_of(a[1], true, false, b)) return not_impl();
  ShmComm* c = comm_of(a[0]);
  if (!c) return PyErr_Occurred() ? nullptr : (PyErr_SetString(PyExc_ValueError, "ccmpi: communicator freed"), nullptr);
  int root = (int)PyLong_AsLong(a[2]);
  if (PyErr_Occurred()) return nullptr;
  if (!guarded([&] { c->bcast(b.ptr(), b.nbytes(), root); })) return nullptr;
  Py_RETURN_NONE;
}

// fallreduce(comm, sbuf, rbuf, op): element type from the buffers' format
PyObject* f_allreduce(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 4, "fallreduce")) return nullptr;
  View s, r;
  if (!view_of(a[1], false, true, s) || !view_of(a[2], true, true, r)) return not_impl();
  const int dt = dtype_of(r);
  if (dt < 0 || dtype_of(s) != dt || s.nbytes() != r.nbytes()) return not_impl();
  ShmComm* c = comm_of(a[0]);
  if (!c) return PyErr_Occurred() ? nullptr : (PyErr_SetString(PyExc_ValueError, "ccmpi: communicator freed"), nullptr);
  int op = (int)PyLong_AsLong(a[3]);
  if (PyErr_Occurred()) return nullptr;
  if (!reduce_supported(dt, op)) return not_impl();
  if (!guarded([&] { c->allreduce(s.ptr(), r.ptr(), r.nbytes() / dtype_size(dt), dt, op); })) return nullptr;
  Py_RETURN_NONE;
}

PyObject* f_allgather(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 3, "fallgather")) return nullptr;
  View s, r;
  if (!view_of(a[1], false, false, s) || !view_of(a[2], true, false, r)) return not_impl();
  ShmComm* c = comm_of(a[0]);
  if (!c) return PyErr_Occurred() ? nullptr : (PyErr_SetString(PyExc_ValueError, "ccmpi: communicator freed"), nullptr);
  if (r.nbytes() != s.nbytes() * (size_t)c->size()) return not_impl();
  if (!guarded([&] { c->allgather(s.ptr(), s.nbytes(), r.ptr()); })) return nullptr;
  Py_RETURN_NONE;
}

PyObject* f_alltoall(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 3, "falltoall")) return nullptr;
  View s, r;
  if (!view_of(a[1], false, false, s) || !view_of(a[2], true, false, r)) return not_impl();
  ShmComm* c = comm_of(a[0]);
  if (!c) return PyErr_Occurred() ? nullptr : (PyErr_SetString(PyExc_ValueError, "ccmpi: communicator freed"), nullptr);
  if (s.nbytes() != r.nbytes() || r.nbytes() % (size_t)c->size()) return not_impl();
  if (!guarded([&] { c->alltoall(s.ptr(), r.nbytes() / c->size(), r.ptr()); })) return nullptr;
  Py_RETURN_NONE;
}

PyObject* f_reduce_scatter_block(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 4, "freduce_scatter_block")) return nullptr;
  View s, r;
  if (!view_of(a[1], false, true, s) || !view_of(a[2], true, true, r)) return not_impl();
  const int dt = dtype_of(r);
  ShmComm* c = comm_of(a[0]);
  if (!c) return PyErr_Occurred() ? nullptr : (PyErr_SetString(PyExc_ValueError, "ccmpi: communicator freed"), nullptr);
  if (dt < 0 || dtype_of(s) != dt || s.nbytes() != r.nbytes() * (size_t)c->size()) return not_impl();
  int op = (int)PyLong_AsLong(a[3]);
  if (PyErr_Occurred()) return nullptr;
  if (!reduce_supported(dt, op)) return not_impl();
  if (!guarded([&] { c->reduce_scatter_block(s.ptr(), r.ptr(), r.nbytes() / dtype_size(dt), dt, op); }))
    return nullptr;
  Py_RETURN_NONE;
}

// ---- the reference's hand-written collectives (p2p_algos.cpp) -------------
// fmy_allreduce(comm, src, dst, op, algo): algo 0 = reduce_bcast, 1 = ring, 2 = rhd
PyObject* f_my_allreduce(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 5, "fmy_allreduce")) return nullptr;
  View s, r;
  if (!view_of(a[1], false, true, s) || !view_of(a[2], true, true, r)) return not_impl();
  const int dt = dtype_of(r);
  if (dt < 0 || dtype_of(s) != dt || s.nbytes() != r.nbytes()) return not_impl();
  ShmComm* c = comm_of(a[0]);
  if (!c) return PyErr_Occurred() ? nullptr : (PyErr_SetString(PyExc_ValueError, "ccmpi: communicator freed"), nullptr);
  int op = (int)PyLong_AsLong(a[3]), algo = (int)PyLong_AsLong(a[4]);
  if (PyErr_Occurred()) return nullptr;
  if (!reduce_supported(dt, op)) return not_impl();
  const size_t count = r.nbytes() / dtype_size(dt);
  bool ok = guarded([&] {
    if (algo == 1)
      c->my_ring_allreduce(s.ptr(), r.ptr(), count, dt, op);
    else if (algo == 2)
      c->my_rhd_allreduce(s.ptr(), r.ptr(), count, dt, op);
    else
      c->my_reduce_bcast(s.ptr(), r.ptr(), count, dt, op);
  });
  if (!ok) return nullptr;
  Py_RETURN_NONE;
}

// fmy_alltoall(comm, src, dst, pairwise)
PyObject* f_my_alltoall(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 4, "fmy_alltoall")) return nullptr;
  View s, r;
  if (!view_of(a[1], false, false, s) || !view_of(a[2], true, false, r)) return not_impl();
  ShmComm* c = comm_of(a[0]);
  if (!c) return PyErr_Occurred() ? nullptr : (PyErr_SetString(PyExc_ValueError, "ccmpi: communicator freed"), nullptr);
  const int pairwise = PyObject_IsTrue(a[3]);
  if (pairwise < 0) return nullptr;
  if (s.nbytes() != r.nbytes() || r.nbytes() % (size_t)c->size()) return not_impl();
  const size_t blk = r.nbytes() / c->size();
  bool ok = guarded([&] {
    if (pairwise)
      c->my_alltoall_pairwise(s.ptr(), r.ptr(), blk);
    else
      c->my_alltoall_nb(s.ptr(), r.ptr(), blk);
  });
  if (!ok) return nullptr;
  Py_RETURN_NONE;
}

// freduce_local(src, dst, op): dst = dst (op) src, element type from the format
PyObject* f_reduce_local(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (!nargs_is(n, 3, "freduce_local")) return nullptr;
  View s, d;
  if (!view_of(a[0], false, true, s) || !view_of(a[1], true, true, d)) return not_impl();
  const int dt = dtype_of(d);
  if (dt < 0 || dtype_of(s) != dt || s.nbytes() != d.nbytes()) return not_impl();
  int op = (int)PyLong_AsLong(a[2]);
  if (PyErr_Occurred()) return nullptr;
  if (!reduce_supported(dt, op)) return not_impl();
  reduce_inplace(d.ptr(), s.ptr(), d.nbytes() / dtype_size(dt), dt, op);
  Py_RETURN_NONE;
}

#define FASTFN(name, fn) {name, reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(fn)), METH_FASTCALL, nullptr}

PyMethodDef g_methods[] = {
    FASTFN("fsend", f_send),
    FASTFN("frecv", f_recv),
    FASTFN("fisend", f_isend),
    FASTFN("firecv", f_irecv),
    FASTFN("fwait", f_wait),
    FASTFN("ftest", f_test),
    FASTFN("fwaitall", f_waitall),
    FASTFN("fsendrecv", f_sendrecv),
    FASTFN("fbarrier", f_barrier),
    FASTFN("fbcast", f_bcast),
    FASTFN("fallreduce", f_allreduce),
    FASTFN("fallgather", f_allgather),
    FASTFN("falltoall", f_alltoall),
    FASTFN("freduce_scatter_block", f_reduce_scatter_block),
    FASTFN("fmy_allreduce", f_my_allreduce),
    FASTFN("fmy_alltoall", f_my_alltoall),
    FASTFN("freduce_local", f_reduce_local),
    {nullptr, nullptr, 0, nullptr},
};

}  // namespace

int register_fastcall(PyObject* module) { return PyModule_AddFunctions(module, g_methods); }

}  // namespace ccmpi
