// pybind11 bindings of the host plane (module `_host`).  The Python layer
// (collective_communication_mpi_amd/mpi.py) builds the mpi4py-compatible API
// on top; this file only moves raw buffers.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "shm_comm.hpp"

namespace py = pybind11;
using namespace ccmpi;

namespace ccmpi {
int register_fastcall(PyObject* module);  // fastcall.cpp
int install_crash_handler(int fd);        // crash.cpp
}

namespace {

struct Buf {
  char* ptr = nullptr;
  size_t nbytes = 0;
};

bool c_contiguous(const py::buffer_info& info) {
  if (info.ndim == 0) return true;
  py::ssize_t expect = info.itemsize;
  for (py::ssize_t d = info.ndim - 1; d >= 0; --d) {
    if (info.shape[d] != 1 && info.strides[d] != expect) return false;
    expect *= info.shape[d];
  }
  return true;
}

Buf get_buf(const py::object& o, bool writable) {
  Buf b;
  if (o.is_none()) return b;
  py::buffer pb = py::reinterpret_borrow<py::buffer>(o);
  py::buffer_info info = pb.request(writable);
  if (!c_contiguous(info))
    throw std::invalid_argument("ccmpi: buffers must be C-contiguous");
  b.ptr = static_cast<char*>(info.ptr);
  b.nbytes = (size_t)info.size * (size_t)info.itemsize;
  return b;
}

py::tuple status_of(const RequestPtr& r) {
  return py::make_tuple(r->st_source, r->st_tag, r->st_count);
}

std::vector<size_t> to_sizes(const std::vector<long long>& v) {
  std::vector<size_t> o(v.size());
  for (size_t i = 0; i < v.size(); ++i) {
    if (v[i] < 0) throw std::invalid_argument("ccmpi: negative count/displacement");
    o[i] = (size_t)v[i];
  }
  return o;
}

}  // namespace

PYBIND11_MODULE(_host, m) {
  m.doc() = "ccmpi host plane: shared-memory intra-node message passing (C++)";
  m.attr("ANY_SOURCE") = ANY_SOURCE;
  m.attr("ANY_TAG") = ANY_TAG;
  m.attr("PROC_NULL") = PROC_NULL;

  if (register_fastcall(m.ptr()) != 0) throw py::error_already_set();
  m.def("wtime", &wtime);
  m.def("p2p_trace", []() { return p2p_trace_take(); }, "phase timestamps of reduce->bcast calls since the last read (CCMPI_P2P_TRACE=1)");
  m.def("install_crash_handler", &install_crash_handler, py::arg("fd") = 2,
        "Print a native backtrace on SIGSEGV/SIGBUS/SIGILL/SIGFPE/SIGABRT, then chain to the previous handler");
  m.def("job_id", &job_id_from_env);
  m.def("dtype_size", &dtype_size);
  m.def("reduce_supported", &reduce_supported);
  m.def("reduce_local", [](py::object src, py::object dst, int dt, int op) {
    Buf s = get_buf(src, false), d = get_buf(dst, true);
    if (s.nbytes != d.nbytes) throw std::invalid_argument("ccmpi: reduce_local size mismatch");
    reduce_inplace(d.ptr, s.ptr, d.nbytes / dtype_size(dt), dt, op);
  });

  py::class_<Request, RequestPtr>(m, "Request")
      .def_property_readonly("complete", [](const Request& r) { return r.complete; })
      .def_property_readonly("status", [](const RequestPtr& r) { return status_of(r); });

  // opaque handle of a started non-blocking collective (nbcoll.cpp)
  py::class_<NbColl, NbCollPtr>(m, "CollRequest")
      .def_property_readonly("done", [](const NbColl& c) { return c.done; });

  py::class_<ShmComm, std::shared_ptr<ShmComm>>(m, "HostComm")
      .def_static("world", &ShmComm::world, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("ptr", [](ShmComm& c) { return reinterpret_cast<uintptr_t>(&c); })
      .def_property_readonly("rank", &ShmComm::rank)
      .def_property_readonly("size", &ShmComm::size)
      .def_property_readonly("name", &ShmComm::name)
      .def_property_readonly("world_ranks", &ShmComm::world_ranks)
      .def_property_readonly("slot_bytes", &ShmComm::slot_bytes)
      .def_property_readonly("ring_bytes", &ShmComm::ring_bytes)
      .def("progress", &ShmComm::progress)
      .def("barrier", &ShmComm::barrier, py::call_guard<py::gil_scoped_release>())
      // ---- point to point ----
      .def("isend", [](ShmComm& c, py::object buf, int dest, int tag) {
        Buf b = get_buf(buf, false);
        py::gil_scoped_release g;
        return c.isend(b.ptr, b.nbytes, dest, tag);
      })
      .def("irecv", [](ShmComm& c, py::object buf, int source, int tag) {
        Buf b = get_buf(buf, true);
        py::gil_scoped_release g;
        return c.irecv(b.ptr, b.nbytes, source, tag);
      })
      .def("wait", [](ShmComm& c, const RequestPtr& r) {
        { py::gil_scoped_release g; c.wait(r); }
        return status_of(r);
      })
      .def("test", [](ShmComm& c, const RequestPtr& r) { return c.test(r); })
      .def("waitall", [](ShmComm& c, const std::vector<RequestPtr>& rs) {
        py::gil_scoped_release g;
        c.waitall(rs);
      })
      .def("waitany", [](ShmComm& c, const std::vector<RequestPtr>& rs) {
        py::gil_scoped_release g;
        return c.waitany(rs);
      })
      .def("send", [](ShmComm& c, py::object buf, int dest, int tag) {
        Buf b = get_buf(buf, false);
        py::gil_scoped_release g;
        c.send(b.ptr, b.nbytes, dest, tag);
      })
      .def("recv", [](ShmComm& c, py::object buf, int source, int tag) {
        Buf b = get_buf(buf, true);
        RequestPtr r;
        { py::gil_scoped_release g; r = c.recv(b.ptr, b.nbytes, source, tag); }
        return status_of(r);
      })
      .def("sendrecv", [](ShmComm& c, py::object sbuf, int dest, int stag, py::object rbuf,
                          int source, int rtag) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        RequestPtr rr;
        { py::gil_scoped_release g; rr = c.sendrecv(s.ptr, s.nbytes, dest, stag, r.ptr, r.nbytes, source, rtag); }
        return status_of(rr);
      })
      .def("probe", [](ShmComm& c, int source, int tag) {
        int s = -1, t = -1;
        size_t n = 0;
        { py::gil_scoped_release g; c.probe(source, tag, &s, &t, &n); }
        return py::make_tuple(s, t, n);
      })
      .def("iprobe", [](ShmComm& c, int source, int tag) -> py::object {
        int s = -1, t = -1;
        size_t n = 0;
        if (!c.iprobe(source, tag, &s, &t, &n)) return py::none();
        return py::make_tuple(s, t, n);
      })
      // ---- non-blocking collectives (None send buffer == IN_PLACE) ----
      .def("ibarrier", [](ShmComm& c) {
        py::gil_scoped_release g;
        return c.ibarrier();
      })
      .def("ibcast", [](ShmComm& c, py::object buf, int root) {
        Buf b = get_buf(buf, true);
        py::gil_scoped_release g;
        return c.ibcast(b.ptr, b.nbytes, root);
      })
      .def("iallreduce", [](ShmComm& c, py::object sbuf, py::object rbuf, int dt, int op) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        if (s.ptr && s.nbytes != r.nbytes) throw std::invalid_argument("ccmpi: Iallreduce buffer size mismatch");
        py::gil_scoped_release g;
        return c.iallreduce(s.ptr, r.ptr, r.nbytes / dtype_size(dt), dt, op);
      })
      .def("iallgather", [](ShmComm& c, py::object sbuf, py::object rbuf) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        if (r.nbytes % c.size()) throw std::invalid_argument("ccmpi: Iallgather receive buffer not divisible by comm size");
        const size_t blk = r.nbytes / c.size();
        if (s.ptr && s.nbytes != blk) throw std::invalid_argument("ccmpi: Iallgather send size != receive block");
        py::gil_scoped_release g;
        return c.iallgather(s.ptr, blk, r.ptr);
      })
      .def("ialltoall", [](ShmComm& c, py::object sbuf, py::object rbuf) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        if (r.nbytes % c.size()) throw std::invalid_argument("ccmpi: Ialltoall buffer not divisible by comm size");
        if (s.ptr && s.nbytes != r.nbytes) throw std::invalid_argument("ccmpi: Ialltoall buffer size mismatch");
        py::gil_scoped_release g;
        return c.ialltoall(s.ptr, r.nbytes / c.size(), r.ptr);
      })
      .def("ireduce_scatter_block", [](ShmComm& c, py::object sbuf, py::object rbuf, int dt, int op) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        const size_t es = dtype_size(dt);
        size_t count;
        if (s.ptr) {
          if (s.nbytes % (es * c.size())) throw std::invalid_argument("ccmpi: Ireduce_scatter_block send count not divisible by comm size");
          count = s.nbytes / es / c.size();
          if (r.nbytes < count * es) throw std::invalid_argument("ccmpi: Ireduce_scatter_block receive buffer too small");
        } else {
          if (r.nbytes % (es * c.size())) throw std::invalid_argument("ccmpi: Ireduce_scatter_block in-place buffer not divisible by comm size");
          count = r.nbytes / es / c.size();
        }
        py::gil_scoped_release g;
        return c.ireduce_scatter_block(s.ptr, r.ptr, count, dt, op);
      })
      .def("nb_test", [](ShmComm& c, const NbCollPtr& r) {
        py::gil_scoped_release g;
        return c.nb_test(r);
      })
      .def("nb_wait", [](ShmComm& c, const NbCollPtr& r) {
        py::gil_scoped_release g;
        c.nb_wait(r);
      })
      .def_property_readonly("nb_active", &ShmComm::nb_active)
      // ---- collectives on raw buffers (None send buffer == IN_PLACE) ----
      .def("bcast", [](ShmComm& c, py::object buf, int root) {
        Buf b = get_buf(buf, true);
        py::gil_scoped_release g;
        c.bcast(b.ptr, b.nbytes, root);
      })
      .def("allreduce", [](ShmComm& c, py::object sbuf, py::object rbuf, int dt, int op) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        if (s.ptr && s.nbytes != r.nbytes) throw std::invalid_argument("ccmpi: Allreduce buffer size mismatch");
        size_t count = r.nbytes / dtype_size(dt);
        py::gil_scoped_release g;
        c.allreduce(s.ptr, r.ptr, count, dt, op);
      })
      .def("reduce", [](ShmComm& c, py::object sbuf, py::object rbuf, int dt, int op, int root) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        size_t count = (s.ptr ? s.nbytes : r.nbytes) / dtype_size(dt);
        if (c.rank() == root && r.nbytes < count * dtype_size(dt))
          throw std::invalid_argument("ccmpi: Reduce receive buffer too small");
        std::vector<char> scratch;
        char* rp = r.ptr;
        if (c.rank() != root || !rp) { scratch.resize(count * dtype_size(dt)); rp = scratch.data(); }
        py::gil_scoped_release g;
        c.reduce(s.ptr, rp, count, dt, op, root);
      })
      .def("reduce_scatter", [](ShmComm& c, py::object sbuf, py::object rbuf,
                                const std::vector<long long>& counts, int dt, int op) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        auto cs = to_sizes(counts);
        py::gil_scoped_release g;
        c.reduce_scatter(s.ptr, r.ptr, cs, dt, op);
      })
      .def("allgatherv", [](ShmComm& c, py::object sbuf, py::object rbuf,
                            const std::vector<long long>& counts, const std::vector<long long>& displs) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        auto cs = to_sizes(counts), ds = to_sizes(displs);
        size_t nb = s.ptr ? s.nbytes : cs.at(c.rank());
        py::gil_scoped_release g;
        c.allgatherv(s.ptr, nb, r.ptr, cs, ds);
      })
      .def("gatherv", [](ShmComm& c, py::object sbuf, py::object rbuf,
                         const std::vector<long long>& counts, const std::vector<long long>& displs, int root) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        auto cs = to_sizes(counts), ds = to_sizes(displs);
        size_t nb = s.ptr ? s.nbytes : (c.rank() == root ? cs.at(c.rank()) : 0);
        py::gil_scoped_release g;
        c.gatherv(s.ptr, nb, r.ptr, cs, ds, root);
      })
      .def("scatterv", [](ShmComm& c, py::object sbuf, const std::vector<long long>& counts,
                          const std::vector<long long>& displs, py::object rbuf, int root) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        auto cs = to_sizes(counts), ds = to_sizes(displs);
        size_t nb = r.ptr ? r.nbytes : 0;
        py::gil_scoped_release g;
        c.scatterv(s.ptr, cs, ds, r.ptr, nb, root);
      })
      .def("alltoall", [](ShmComm& c, py::object sbuf, py::object rbuf) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        if (r.nbytes % c.size()) throw std::invalid_argument("ccmpi: Alltoall buffer not divisible by comm size");
        if (s.ptr && s.nbytes != r.nbytes) throw std::invalid_argument("ccmpi: Alltoall buffer size mismatch");
        py::gil_scoped_release g;
        c.alltoall(s.ptr, r.nbytes / c.size(), r.ptr);
      })
      .def("alltoallv", [](ShmComm& c, py::object sbuf, const std::vector<long long>& sc,
                           const std::vector<long long>& sd, py::object rbuf,
                           const std::vector<long long>& rc, const std::vector<long long>& rd) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        auto a = to_sizes(sc), b = to_sizes(sd), x = to_sizes(rc), y = to_sizes(rd);
        py::gil_scoped_release g;
        c.alltoallv(s.ptr, a, b, r.ptr, x, y);
      })
      .def("scan", [](ShmComm& c, py::object sbuf, py::object rbuf, int dt, int op, bool exclusive) {
        Buf s = get_buf(sbuf, false), r = get_buf(rbuf, true);
        py::gil_scoped_release g;
        c.scan(s.ptr, r.ptr, r.nbytes / dtype_size(dt), dt, op, exclusive);
      })
      .def("split", [](ShmComm& c, int color, int key) -> py::object {
        std::shared_ptr<ShmComm> r;
        { py::gil_scoped_release g; r = c.split(color, key); }
        if (!r) return py::none();
        return py::cast(r);
      })
      // ---- variable-size byte collectives for pickled objects ----
      .def("allgather_bytes", [](ShmComm& c, py::bytes data) {
        std::string s = data;
        int p = c.size();
        std::vector<int64_t> sizes(p);
        int64_t mine = (int64_t)s.size();
        std::vector<size_t> counts(p), displs(p);
        std::string out;
        {
          py::gil_scoped_release g;
          c.allgather(&mine, 8, sizes.data());
          size_t tot = 0;
          for (int i = 0; i < p; ++i) { counts[i] = (size_t)sizes[i]; displs[i] = tot; tot += counts[i]; }
          out.resize(tot);
          c.allgatherv(s.data(), s.size(), out.data(), counts, displs);
        }
        py::list l;
        for (int i = 0; i < p; ++i) l.append(py::bytes(out.data() + displs[i], counts[i]));
        return l;
      })
      .def("alltoall_bytes", [](ShmComm& c, const std::vector<std::string>& parts) {
        int p = c.size();
        if ((int)parts.size() != p) throw std::invalid_argument("ccmpi: alltoall needs one object per rank");
        std::vector<int64_t> ss(p), rs(p);
        for (int i = 0; i < p; ++i) ss[i] = (int64_t)parts[i].size();
        std::vector<size_t> sc(p), sd(p), rc(p), rd(p);
        std::string sbuf, rbuf;
        {
          py::gil_scoped_release g;
          c.alltoall(ss.data(), 8, rs.data());
          size_t t = 0;
          for (int i = 0; i < p; ++i) { sc[i] = (size_t)ss[i]; sd[i] = t; t += sc[i]; }
          sbuf.reserve(t);
          for (auto& x : parts) sbuf += x;
          t = 0;
          for (int i = 0; i < p; ++i) { rc[i] = (size_t)rs[i]; rd[i] = t; t += rc[i]; }
          rbuf.resize(t);
          c.alltoallv(sbuf.data(), sc, sd, rbuf.data(), rc, rd);
        }
        py::list l;
        for (int i = 0; i < p; ++i) l.append(py::bytes(rbuf.data() + rd[i], rc[i]));
        return l;
      })
      .def("bcast_bytes", [](ShmComm& c, py::object data, int root) {
        std::string s;
        if (c.rank() == root) s = py::cast<std::string>(data);
        {
          py::gil_scoped_release g;
          int64_t n = (int64_t)s.size();
          c.bcast(&n, 8, root);
          s.resize((size_t)n);
          c.bcast(s.data(), s.size(), root);
        }
        return py::bytes(s);
      })
      .def("gather_bytes", [](ShmComm& c, py::bytes data, int root) -> py::object {
        std::string s = data;
        int p = c.size();
        std::vector<int64_t> sizes(p);
        int64_t mine = (int64_t)s.size();
        std::vector<size_t> counts(p), displs(p);
        std::string out;
        {
          py::gil_scoped_release g;
          c.allgather(&mine, 8, sizes.data());
          size_t tot = 0;
          for (int i = 0; i < p; ++i) { counts[i] = (size_t)sizes[i]; displs[i] = tot; tot += counts[i]; }
          if (c.rank() == root) out.resize(tot);
          c.gatherv(s.data(), s.size(), c.rank() == root ? out.data() : nullptr, counts, displs, root);
        }
        if (c.rank() != root) return py::none();
        py::list l;
        for (int i = 0; i < p; ++i) l.append(py::bytes(out.data() + displs[i], counts[i]));
        return l;
      })
      .def("scatter_bytes", [](ShmComm& c, py::object parts, int root) {
        int p = c.size();
        std::vector<std::string> ps;
        if (c.rank() == root) {
          ps = py::cast<std::vector<std::string>>(parts);
          if ((int)ps.size() != p) throw std::invalid_argument("ccmpi: scatter needs one object per rank");
        }
        std::string out;
        {
          py::gil_scoped_release g;
          std::vector<int64_t> sizes(p), mine(1);
          if (c.rank() == root) for (int i = 0; i < p; ++i) sizes[i] = (int64_t)ps[i].size();
          c.bcast(sizes.data(), 8 * (size_t)p, root);
          std::vector<size_t> counts(p), displs(p);
          size_t t = 0;
          for (int i = 0; i < p; ++i) { counts[i] = (size_t)sizes[i]; displs[i] = t; t += counts[i]; }
          std::string sbuf;
          if (c.rank() == root) { sbuf.reserve(t); for (auto& x : ps) sbuf += x; }
          out.resize(counts[c.rank()]);
          c.scatterv(sbuf.data(), counts, displs, out.data(), out.size(), root);
        }
        return py::bytes(out);
      });
}
