// pybind11 bindings of the device plane (module `_device`).  Pointers and
// streams cross the boundary as integers (tensor.data_ptr(), stream.cuda_stream)
// so the module does not link libtorch.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <memory>

#include "device_comm.hpp"
#include "ops.hpp"
#include "symheap.hpp"

namespace py = pybind11;
using namespace ccmpi::dev;

namespace {
// Minimal DLPack (v0.8 ABI) to hand symmetric-heap blocks to torch with a
// deleter that returns the block to the heap when the tensor's storage dies.
struct DLDevice { int32_t device_type; int32_t device_id; };
struct DLDataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct DLTensor {
  void* data; DLDevice device; int32_t ndim; DLDataType dtype; int64_t* shape; int64_t* strides; uint64_t byte_offset;
};
struct DLManagedTensor { DLTensor dl_tensor; void* manager_ctx; void (*deleter)(DLManagedTensor*); };
constexpr int32_t kDLROCM = 10;
constexpr uint8_t kDLUInt = 1;

struct BlockCtx {
  std::shared_ptr<SymHeap> heap;
  uint64_t ptr;
  int64_t shape[1];
};

void block_deleter(DLManagedTensor* t) {  // may run without the GIL: no Python here
  auto* c = static_cast<BlockCtx*>(t->manager_ctx);
  c->heap->release(c->ptr);
  delete c;
  delete t;
}

void capsule_destructor(PyObject* cap) {  // only when torch never consumed the capsule
  if (PyCapsule_IsValid(cap, "dltensor")) {
    auto* t = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
    if (t && t->deleter) t->deleter(t);
  }
}

py::object heap_block(const std::shared_ptr<SymHeap>& heap, uint64_t bytes, int device) {
  const uint64_t ptr = heap->alloc(bytes);
  if (!ptr) return py::none();
  auto* c = new BlockCtx{heap, ptr, {(int64_t)bytes}};
  auto* t = new DLManagedTensor{};
  t->dl_tensor.data = reinterpret_cast<void*>(ptr);
  t->dl_tensor.device = {kDLROCM, device};
  t->dl_tensor.ndim = 1;
  t->dl_tensor.dtype = {kDLUInt, 8, 1};
  t->dl_tensor.shape = c->shape;
  t->dl_tensor.strides = nullptr;
  t->dl_tensor.byte_offset = 0;
  t->manager_ctx = c;
  t->deleter = block_deleter;
  return py::reinterpret_steal<py::object>(PyCapsule_New(t, "dltensor", capsule_destructor));
}
}  // namespace

PYBIND11_MODULE(_device, m) {
  m.doc() = "ccmpi device plane: hand-written CDNA4 collectives + kernels (HIP, gfx950)";
  m.attr("ALGO_ONESHOT") = (int)ALGO_ONESHOT;
  m.attr("ALGO_TWOSHOT") = (int)ALGO_TWOSHOT;
  m.attr("ALGO_REDUCE_BCAST") = (int)ALGO_REDUCE_BCAST;
  m.attr("ALGO_TWOSHOT_PUSH") = (int)ALGO_TWOSHOT_PUSH;
  m.attr("ALGO_RING") = (int)ALGO_RING;
  m.attr("ALGO_RHD") = (int)ALGO_RHD;
  m.attr("ALGO_LL") = (int)ALGO_LL;
  m.attr("ALGO_TWOSHOT_FANOUT") = (int)ALGO_TWOSHOT_FANOUT;
  m.attr("ALGO_TWOSHOT_FANOUT_LDS") = (int)ALGO_TWOSHOT_FANOUT_LDS;
  m.attr("A2A_PULL") = (int)A2A_PULL;
  m.attr("A2A_PUSH") = (int)A2A_PUSH;
  m.attr("A2A_PAIRWISE") = (int)A2A_PAIRWISE;
  m.attr("MAX_RINGS") = kMaxRings;
  m.def("ring_slot_bytes", &DeviceComm::ring_slot_bytes);
  m.attr("MAX_RANKS") = kMaxRanks;
  m.attr("MAX_BLOCKS") = kMaxBlocks;
  m.def("reduce_supported", &device_reduce_supported);
  m.def("rccl_unique_id", []() { return py::bytes(DeviceComm::rccl_unique_id()); });

  py::class_<SymHeap, std::shared_ptr<SymHeap>>(m, "SymHeap")
      .def(py::init([]() { return std::make_shared<SymHeap>(); }))
      .def("add_arena", &SymHeap::add_arena)
      .def("alloc", &SymHeap::alloc)
      .def("release", &SymHeap::release)
      // DLPack capsule of a fresh `bytes`-long uint8 block on `device` (None when full)
      .def("block", [](const std::shared_ptr<SymHeap>& h, uint64_t bytes, int device) { return heap_block(h, bytes, device); })
      .def_property_readonly("used_bytes", &SymHeap::used_bytes)
      .def_property_readonly("capacity", &SymHeap::capacity)
      .def_property_readonly("largest_free", &SymHeap::largest_free)
      .def_property_readonly("live_blocks", &SymHeap::live_blocks);

  py::class_<DeviceComm>(m, "DeviceComm")
      .def(py::init<int, int, int, uint64_t>(), py::arg("rank"), py::arg("size"), py::arg("device"),
           py::arg("scratch_bytes") = 0)
      .def_property_readonly("rank", &DeviceComm::rank)
      .def_property_readonly("size", &DeviceComm::size)
      .def_property_readonly("device", &DeviceComm::device)
      .def("signal_handle", [](const DeviceComm& d) { return py::bytes(d.signal_handle()); })
      .def("connect", [](DeviceComm& d, const std::vector<std::string>& hs) { d.connect(hs); })
      .def("export_range", [](const DeviceComm& d, uint64_t ptr) {
        auto r = d.export_range(ptr);
        return py::make_tuple(py::bytes(r.first), r.second);
      })
      .def("add_segment", &DeviceComm::add_segment)
      .def("export_alloc", [](const DeviceComm& d, uint64_t ptr) {
        // (IPC handle bytes, allocation base, allocation bytes) of the allocation holding ptr
        hipDeviceptr_t base = nullptr;
        size_t sz = 0;
        CCMPI_HIP_CHECK(hipMemGetAddressRange(&base, &sz, reinterpret_cast<hipDeviceptr_t>(ptr)));
        auto r = d.export_range((uint64_t)base);
        return py::make_tuple(py::bytes(r.first), (uint64_t)base, (uint64_t)sz);
      })
      .def_static("alloc_id", [](uint64_t ptr) -> uint64_t {
        // the driver's unique id of the allocation holding ptr (0 if unknown): a range
        // freed and reallocated at the same address gets a new id
        unsigned long long id = 0;
        if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, reinterpret_cast<hipDeviceptr_t>(ptr)) !=
            hipSuccess) {
          (void)hipGetLastError();
          return 0;
        }
        return (uint64_t)id;
      })
      .def("set_segment", [](DeviceComm& d, int s, uint64_t ptr, uint64_t bytes, const std::vector<py::bytes>& hs,
                             const std::vector<uint64_t>& offs, const std::vector<py::bytes>& ks) {
        std::vector<std::string> h(hs.begin(), hs.end()), k(ks.begin(), ks.end());
        return d.set_segment(s, ptr, bytes, h, offs, k);
      })
      .def("clear_segment", &DeviceComm::clear_segment)
      .def_property_readonly("num_segments", &DeviceComm::num_segments)
      .def("find", [](const DeviceComm& d, uint64_t ptr, uint64_t n) {
        uint64_t off = 0;
        int s = d.find(ptr, n, &off);
        return py::make_tuple(s, off);
      })
      .def_property_readonly("scratch_bytes", &DeviceComm::scratch_bytes)
      .def("allreduce", &DeviceComm::allreduce, py::call_guard<py::gil_scoped_release>())
      .def("allreduce_to_local", &DeviceComm::allreduce_to_local, py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter", &DeviceComm::reduce_scatter, py::call_guard<py::gil_scoped_release>())
      .def("allgather", &DeviceComm::allgather, py::arg("inp"), py::arg("out"), py::arg("bytes_per_rank"),
           py::arg("stream"), py::arg("max_blocks"), py::arg("symmetric"), py::arg("mode") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("alltoallv_dev", &DeviceComm::alltoallv_dev, py::call_guard<py::gil_scoped_release>())
      .def("alltoallv", &DeviceComm::alltoallv, py::call_guard<py::gil_scoped_release>())
      .def("alltoall", &DeviceComm::alltoall, py::arg("inp"), py::arg("out"), py::arg("bytes_per_peer"),
           py::arg("stream"), py::arg("max_blocks"), py::arg("symmetric"), py::arg("mode") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("bcast", &DeviceComm::bcast, py::arg("buf"), py::arg("nbytes"), py::arg("root"), py::arg("stream"),
           py::arg("max_blocks"), py::arg("symmetric"), py::arg("mode") = 0, py::call_guard<py::gil_scoped_release>())
      .def("local_reduce", &DeviceComm::local_reduce, py::call_guard<py::gil_scoped_release>())
      .def("allgather_lastaxis", &DeviceComm::allgather_lastaxis, py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter_lastaxis", &DeviceComm::reduce_scatter_lastaxis, py::call_guard<py::gil_scoped_release>())
      .def("rccl_init", [](DeviceComm& d, py::bytes uid) {
        std::string u = uid;
        py::gil_scoped_release g;
        d.rccl_init(u);
      })
      .def_property_readonly("rccl_ready", &DeviceComm::rccl_ready)
      .def("rccl_register_segments", &DeviceComm::rccl_register_segments, py::call_guard<py::gil_scoped_release>())
      .def("rccl_split_from", [](DeviceComm& d, DeviceComm* parent, int color, int key) {
        py::gil_scoped_release g;
        d.rccl_split_from(parent, color, key);
      })
      .def_static("rccl_split_nocolor", [](DeviceComm* parent) {
        py::gil_scoped_release g;
        // a parent rank that joins no child still takes part in the split
        DeviceComm::rccl_split_leave(parent);
      })
      .def("rccl_allreduce", &DeviceComm::rccl_allreduce, py::call_guard<py::gil_scoped_release>())
      .def("rccl_reduce_scatter", &DeviceComm::rccl_reduce_scatter, py::call_guard<py::gil_scoped_release>())
      .def("rccl_allgather", &DeviceComm::rccl_allgather, py::call_guard<py::gil_scoped_release>())
      .def("rccl_alltoall", &DeviceComm::rccl_alltoall, py::call_guard<py::gil_scoped_release>())
      .def("rccl_bcast", &DeviceComm::rccl_bcast, py::call_guard<py::gil_scoped_release>())
      .def("p2p_pairwise_alltoall", &DeviceComm::p2p_pairwise_alltoall, py::call_guard<py::gil_scoped_release>())
      .def("error_code", &DeviceComm::error_code, py::call_guard<py::gil_scoped_release>())
      .def("clear_error", &DeviceComm::clear_error)
      .def("poll_error", &DeviceComm::poll_error)
      .def("reset_state", &DeviceComm::reset_state, py::call_guard<py::gil_scoped_release>())
      .def("set_inbox", &DeviceComm::set_inbox)
      .def("ll_alloc", [](DeviceComm& d, uint64_t max_bytes) { return py::bytes(d.ll_alloc(max_bytes)); })
      .def("fused_alloc", [](DeviceComm& d) { return py::bytes(d.fused_alloc()); })
      .def("fused_connect", [](DeviceComm& d, const std::vector<std::string>& hs) { d.fused_connect(hs); })
      .def("set_fused_inbox", &DeviceComm::set_fused_inbox)
      .def_property_readonly("fused_inbox_bytes", &DeviceComm::fused_inbox_bytes)
      .def_property_readonly("fused_ready", &DeviceComm::fused_ready)
      .def("code_of", [](DeviceComm& d, uint64_t ptr, uint64_t n) { return d.code_of_public(ptr, n); })
      .def("gemm_rowpar", &DeviceComm::gemm_rowpar, py::call_guard<py::gil_scoped_release>())
      .def("gemm_push_rowpar", &DeviceComm::gemm_push_rowpar, py::call_guard<py::gil_scoped_release>())
      .def("push_targets", &DeviceComm::push_targets)
      .def("inbox_to_local", &DeviceComm::inbox_to_local, py::call_guard<py::gil_scoped_release>())
      .def("inbox_mean", &DeviceComm::inbox_mean, py::call_guard<py::gil_scoped_release>())
      .def("ll_connect", [](DeviceComm& d, const std::vector<std::string>& hs) { d.ll_connect(hs); })
      .def_property_readonly("ll_max_bytes", &DeviceComm::ll_max_bytes)
      .def_property_readonly("inbox_bytes", &DeviceComm::inbox_bytes)
      .def("set_timeout_seconds", &DeviceComm::set_timeout_seconds)
      .def("set_copy_engine", &DeviceComm::set_copy_engine)
      .def("set_rings", &DeviceComm::set_rings)
      .def("set_debug_stamps", &DeviceComm::set_debug_stamps)
      .def_property_readonly("rings", &DeviceComm::rings);

  register_ops(m);
}
