// Python bindings of the GPU runtime: device helpers, gfx950 kernels on raw
// device pointers, pinned host buffers, and the RCCL data engine.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>

#include "core/crc32c.h"
#include "core/fp8.h"
#include "gpu/gpu_api.h"
#include "gpu/hip_backend.h"
#include "kernels/kernels.h"

namespace py = pybind11;
using namespace dissem;

namespace {

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

hipStream_t as_stream(uint64_t s) { return reinterpret_cast<hipStream_t>(s); }

// Per-device scratch for synchronous CRC calls from Python.
struct Scratch {
  void* ws = nullptr;
  size_t ws_bytes = 0;
  uint32_t* out = nullptr;  // pinned
  size_t out_n = 0;
};
std::mutex g_scratch_mu;
std::map<int, Scratch> g_scratch;

std::vector<uint32_t> crc_chunks_sync(uint64_t ptr, int64_t bytes, int64_t chunk, uint64_t stream) {
  int dev = 0;
  check(hipGetDevice(&dev), "hipGetDevice");
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  Scratch& s = g_scratch[dev];
  size_t need = kern::crc32c_workspace_bytes(bytes, chunk);
  if (s.ws_bytes < need) {
    if (s.ws) check(hipFree(s.ws), "hipFree");
    check(hipMalloc(&s.ws, need), "hipMalloc");
    check(hipMemset(s.ws, 0, need), "hipMemset");  // fold words: zeroed once (kernels.h)
    s.ws_bytes = need;
  }
  size_t n = size_t(bytes > 0 ? (bytes + chunk - 1) / chunk : 0);
  if (s.out_n < n) {
    if (s.out) check(hipHostFree(s.out), "hipHostFree");
    check(hipHostMalloc(reinterpret_cast<void**>(&s.out), std::max<size_t>(n, 1) * 4, hipHostMallocMapped), "hipHostMalloc");
    s.out_n = n;
  }
  uint32_t* dout = nullptr;
  check(hipHostGetDevicePointer(reinterpret_cast<void**>(&dout), s.out, 0), "hipHostGetDevicePointer");
  check(kern::crc32c_chunks(reinterpret_cast<const void*>(ptr), bytes, chunk, dout, s.ws, as_stream(stream)),
        "crc32c_chunks");
  check(hipStreamSynchronize(as_stream(stream)), "hipStreamSynchronize");
  return std::vector<uint32_t>(s.out, s.out + n);
}

}  // namespace

void register_gpu_bindings(PyObject* module) {
  py::module_ m = py::reinterpret_borrow<py::module_>(module);

  // ---- host CRC32C reference + GF(2) helpers (tests compare kernels against these)
  m.def("crc32c", [](py::buffer b, uint32_t crc) {
    py::buffer_info info = b.request();
    return crc32c(info.ptr, size_t(info.size * info.itemsize), crc);
  }, py::arg("data"), py::arg("crc") = 0);
  m.def("crc32c_shift", &crc32c_shift);
  m.def("crc32c_multmodp", &crc32c_multmodp);
  m.def("fill_random_host", [](int64_t n, uint64_t seed, int64_t offset) {
    std::string out(size_t(n), '\0');
    {
      py::gil_scoped_release nogil;
      kern::fill_random_host(out.data(), n, seed, offset);
    }
    return py::bytes(out);
  }, py::arg("n"), py::arg("seed"), py::arg("offset") = 0);

  // ---- device helpers
  m.def("device_count", [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("set_device", [](int d) { check(hipSetDevice(d), "hipSetDevice"); });
  // Pairwise GPU links (SURVEY C4's topology map): (i, j, link, hops, p2p) with
  // link "xgmi" / "pcie" / "other" from hipExtGetLinkTypeAndHopCount.
  m.def("gpu_topology", [] {
    int n = 0;
    check(hipGetDeviceCount(&n), "hipGetDeviceCount");
    py::list out;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        if (i == j) continue;
        uint32_t type = 0, hops = 0;
        const char* link = "other";
        if (hipExtGetLinkTypeAndHopCount(i, j, &type, &hops) == hipSuccess) {
          if (type == 4) link = "xgmi";       // HSA_AMD_LINK_INFO_TYPE_XGMI
          else if (type == 2) link = "pcie";  // HSA_AMD_LINK_INFO_TYPE_PCIE
        }
        int p2p = 0;
        (void)hipDeviceCanAccessPeer(&p2p, i, j);
        out.append(py::make_tuple(i, j, std::string(link), hops, bool(p2p)));
      }
    return out;
  });
  // Regression probe (round 3): the first CRC of a new chunk size must not
  // wait for other streams. A blocking stream holds a kernel that spins until
  // the host releases it (an RCCL kernel waiting on a peer); meanwhile a CRC of
  // a never-seen size is launched on another stream. Returns (host ms of that
  // launch call, spin iterations, crc, spin stream drained). Before the fix the
  // launch blocked in a null-stream hipMemcpy until the spin ran out.
  m.def("crc_launch_beside_blocked_stream", [](int64_t bytes, uint64_t max_iters) {
    py::gil_scoped_release nogil;
    hipStream_t blocked = nullptr, work = nullptr;
    check(hipStreamCreate(&blocked), "hipStreamCreate");  // default flags: blocking, like the lanes
    check(hipStreamCreateWithFlags(&work, hipStreamNonBlocking), "hipStreamCreateWithFlags");
    uint32_t* flag = nullptr;
    uint32_t *flag_dev = nullptr, *out = nullptr;
    uint64_t* iters = nullptr;
    check(hipHostMalloc(reinterpret_cast<void**>(&flag), 4, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
    *flag = 0;
    check(hipHostGetDevicePointer(reinterpret_cast<void**>(&flag_dev), flag, 0), "hipHostGetDevicePointer");
    check(hipMalloc(reinterpret_cast<void**>(&iters), 8), "hipMalloc");
    check(hipMalloc(reinterpret_cast<void**>(&out), 4), "hipMalloc");
    uint8_t* data = nullptr;
    check(hipMalloc(reinterpret_cast<void**>(&data), size_t(bytes)), "hipMalloc");
    check(kern::fill_random(data, bytes, 7, work), "fill");
    check(hipStreamSynchronize(work), "sync");
    void* ws = nullptr;
    check(hipMalloc(&ws, kern::crc32c_workspace_bytes(bytes, bytes)), "hipMalloc");
    check(hipMemsetAsync(ws, 0, kern::crc32c_workspace_bytes(bytes, bytes), work), "hipMemsetAsync");
    check(hipStreamSynchronize(work), "sync");
    check(kern::spin_until(flag_dev, max_iters, iters, blocked), "spin");
    const auto t0 = std::chrono::steady_clock::now();
    check(kern::crc32c_chunks(data, bytes, bytes, out, ws, work), "crc32c_chunks");
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    __atomic_store_n(flag, 1u, __ATOMIC_RELEASE);
    check(hipStreamSynchronize(blocked), "sync blocked");
    check(hipStreamSynchronize(work), "sync work");
    uint32_t crc = 0;
    uint64_t it = 0;
    check(hipMemcpy(&crc, out, 4, hipMemcpyDeviceToHost), "copy");
    check(hipMemcpy(&it, iters, 8, hipMemcpyDeviceToHost), "copy");
    (void)hipFree(ws);
    (void)hipFree(data);
    (void)hipFree(out);
    (void)hipFree(iters);
    (void)hipHostFree(flag);
    (void)hipStreamDestroy(blocked);
    (void)hipStreamDestroy(work);
    return std::make_tuple(ms, it, crc);
  }, py::arg("bytes"), py::arg("max_iters") = 600000);
  m.def("device_synchronize", [] {
    py::gil_scoped_release nogil;
    check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  });
  m.def("device_malloc", [](int64_t n) {
    void* p = nullptr;
    check(hipMalloc(&p, size_t(n)), "hipMalloc");
    return reinterpret_cast<uint64_t>(p);
  });
  m.def("device_free", [](uint64_t p) { check(hipFree(reinterpret_cast<void*>(p)), "hipFree"); });
  m.def("memcpy", [](uint64_t dst, uint64_t src, int64_t n, uint64_t stream) {
    py::gil_scoped_release nogil;
    check(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<void*>(src), size_t(n), hipMemcpyDefault,
                         as_stream(stream)),
          "hipMemcpyAsync");
    check(hipStreamSynchronize(as_stream(stream)), "hipStreamSynchronize");
  }, py::arg("dst"), py::arg("src"), py::arg("n"), py::arg("stream") = 0);
  m.def("memset", [](uint64_t dst, int v, int64_t n, uint64_t stream) {
    check(hipMemsetAsync(reinterpret_cast<void*>(dst), v, size_t(n), as_stream(stream)), "hipMemsetAsync");
  }, py::arg("dst"), py::arg("value"), py::arg("n"), py::arg("stream") = 0);
  m.def("mem_info", [] {
    size_t f = 0, t = 0;
    check(hipMemGetInfo(&f, &t), "hipMemGetInfo");
    return py::make_tuple(f, t);
  });

  // ---- pinned host memory as a HostBuffer usable by LayerSrc
  py::class_<HostBuffer, std::shared_ptr<HostBuffer>>(m, "HostBuffer")
      .def_static("pinned", [](int64_t n) {
        py::gil_scoped_release nogil;
        return alloc_pinned(n);
      })
      .def_static("malloc", [](int64_t n) { return HostBuffer::alloc(n, true); })
      // Node-shared host memory (POSIX shm): one process creates `name`, the
      // others of the node map it; `pin` registers the mapping with HIP in this
      // process (page-locked, DMA-able by this rank's GPU over its own PCIe).
      // The creator removes the name when its buffer is released (unlink early
      // with shared_unlink once every process has mapped it).
      .def_static("shared", [](const std::string& name, int64_t n, bool create, bool pin) {
        py::gil_scoped_release nogil;
        const std::string nm = name.empty() || name[0] != '/' ? "/" + name : name;
        int fd = shm_open(nm.c_str(), O_RDWR | (create ? O_CREAT | O_EXCL : 0), 0600);
        if (fd < 0) {
          const int e = errno;
          throw std::runtime_error("shm_open " + nm + ": " + strerror(e) +
                                   (e == EEXIST ? " (left by an earlier run that did not finish: remove /dev/shm" + nm +
                                                      " and the run's other /dev/shm/dld_* segments)"
                                                : ""));
        }
        if (create && ftruncate(fd, off_t(n)) != 0) {
          const int e = errno;
          close(fd);
          shm_unlink(nm.c_str());
          throw std::runtime_error("ftruncate " + nm + ": " + strerror(e));
        }
        struct stat stt;
        if (fstat(fd, &stt) != 0 || stt.st_size < n) {
          close(fd);
          throw std::runtime_error("shared buffer " + nm + " is smaller than requested");
        }
        void* p = mmap(nullptr, size_t(n), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED) throw std::runtime_error("mmap " + nm + ": " + strerror(errno));
        if (pin) {
          hipError_t e = hipHostRegister(p, size_t(n), hipHostRegisterDefault);
          if (e != hipSuccess) {
            munmap(p, size_t(n));
            throw std::runtime_error("hipHostRegister " + nm + ": " + hipGetErrorString(e));
          }
        }
        auto owner = std::shared_ptr<void>(p, [n, pin, create, nm](void* q) {
          if (pin) (void)hipHostUnregister(q);
          munmap(q, size_t(n));
          if (create) shm_unlink(nm.c_str());
        });
        return HostBuffer::wrap(static_cast<uint8_t*>(p), n, owner);
      }, py::arg("name"), py::arg("size"), py::arg("create"), py::arg("pin") = true)
      .def_static("shared_exists", [](const std::string& name) {
        const std::string nm = name.empty() || name[0] != '/' ? "/" + name : name;
        int fd = shm_open(nm.c_str(), O_RDONLY, 0);
        if (fd < 0) return false;
        close(fd);
        return true;
      })
      .def_static("shared_unlink", [](const std::string& name) {
        const std::string nm = name.empty() || name[0] != '/' ? "/" + name : name;
        return shm_unlink(nm.c_str()) == 0;
      })
      .def_property_readonly("ptr", [](const HostBuffer& b) { return reinterpret_cast<uint64_t>(b.ptr); })
      .def_property_readonly("size", [](const HostBuffer& b) { return b.size; })
      .def("view", [](HostBuffer& b) {
        return py::memoryview::from_memory(b.ptr, py::ssize_t(b.size), false);
      })
      .def("bytes", [](const HostBuffer& b, int64_t off, int64_t n) {
        if (n < 0) n = b.size - off;
        return py::bytes(reinterpret_cast<const char*>(b.ptr + off), size_t(n));
      }, py::arg("off") = 0, py::arg("n") = -1);
  m.def("layer_src_from_buffer", [](std::shared_ptr<HostBuffer> b, int64_t rate, SourceType st) {
    LayerSrc s;
    s.host = std::move(b);
    s.data_size = s.host->size;
    s.meta = LayerMeta{Location::Inmem, rate, st, s.data_size};
    return s;
  }, py::arg("buffer"), py::arg("limit_rate") = 0, py::arg("source_type") = SourceType::Mem);
  m.def("layer_src_device", [](uint64_t dev_ptr, int64_t size) {
    LayerSrc s;
    s.dev = reinterpret_cast<uint8_t*>(dev_ptr);
    s.data_size = size;
    s.meta = LayerMeta{Location::Device, 0, SourceType::Device, size};
    return s;
  });

  // ---- kernels on raw device pointers (stream = hipStream_t as int, 0 = null stream)
  m.def("fill_random", [](uint64_t ptr, int64_t n, uint64_t seed, uint64_t stream) {
    check(kern::fill_random(reinterpret_cast<void*>(ptr), n, seed, as_stream(stream)), "fill_random");
  }, py::arg("ptr"), py::arg("nbytes"), py::arg("seed"), py::arg("stream") = 0);
  m.def("crc32c_chunks", [](uint64_t ptr, int64_t n, int64_t chunk, uint64_t stream) {
    py::gil_scoped_release nogil;
    return crc_chunks_sync(ptr, n, chunk, stream);
  }, py::arg("ptr"), py::arg("nbytes"), py::arg("chunk_bytes"), py::arg("stream") = 0);
  // Asynchronous forms take a caller-owned workspace of the size the
  // *_workspace_bytes helper names, zeroed once before its first use (every
  // launch leaves it zeroed). `cus`: CUs the stream may use (0: all).
  m.def("crc32c_chunks_async", [](uint64_t ptr, int64_t n, int64_t chunk, uint64_t out_dev, uint64_t ws,
                                  uint64_t stream, int cus) {
    check(kern::crc32c_chunks(reinterpret_cast<const void*>(ptr), n, chunk, reinterpret_cast<uint32_t*>(out_dev),
                              reinterpret_cast<void*>(ws), as_stream(stream), cus),
          "crc32c_chunks");
  }, py::arg("ptr"), py::arg("nbytes"), py::arg("chunk_bytes"), py::arg("out"), py::arg("workspace"),
     py::arg("stream") = 0, py::arg("cus") = 0);
  m.def("crc32c_workspace_bytes", &kern::crc32c_workspace_bytes);
  m.def("crc32c_batch_workspace_bytes", [] { return kern::crc32c_batch_workspace_bytes(); });
  m.def("crc32c_batch_max", [] { return kern::kCrcBatchMax; });
  // Batched CRC of independent device buffers [(ptr, nbytes), ...] (synchronous).
  m.def("crc32c_batch", [](const std::vector<std::pair<uint64_t, int64_t>>& bufs, uint64_t stream, int cus) {
    py::gil_scoped_release nogil;
    if (bufs.size() > size_t(kern::kCrcBatchMax)) throw std::invalid_argument("too many buffers for one batch");
    void* ws = nullptr;
    uint32_t *host = nullptr, *dev = nullptr;
    check(hipMalloc(&ws, kern::crc32c_batch_workspace_bytes()), "hipMalloc");
    check(hipMemset(ws, 0, kern::crc32c_batch_workspace_bytes()), "hipMemset");
    check(hipHostMalloc(reinterpret_cast<void**>(&host), std::max<size_t>(bufs.size(), 1) * 4, hipHostMallocMapped),
          "hipHostMalloc");
    check(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev), host, 0), "hipHostGetDevicePointer");
    std::vector<kern::CrcItem> items;
    for (size_t i = 0; i < bufs.size(); ++i)
      items.push_back(kern::CrcItem{reinterpret_cast<const void*>(bufs[i].first), bufs[i].second, dev + i});
    hipError_t e = kern::crc32c_batch(items.data(), int(items.size()), ws, as_stream(stream), cus);
    if (e == hipSuccess) e = hipStreamSynchronize(as_stream(stream));
    std::vector<uint32_t> out(host, host + bufs.size());
    (void)hipFree(ws);
    (void)hipHostFree(host);
    check(e, "crc32c_batch");
    return out;
  }, py::arg("buffers"), py::arg("stream") = 0, py::arg("cus") = 0);
  m.def("crc32c_batch_async", [](const std::vector<std::pair<uint64_t, int64_t>>& bufs, uint64_t out_dev, uint64_t ws,
                                 uint64_t stream, int cus) {
    if (bufs.size() > size_t(kern::kCrcBatchMax)) throw std::invalid_argument("too many buffers for one batch");
    std::vector<kern::CrcItem> items;
    for (size_t i = 0; i < bufs.size(); ++i)
      items.push_back(kern::CrcItem{reinterpret_cast<const void*>(bufs[i].first), bufs[i].second,
                                    reinterpret_cast<uint32_t*>(out_dev) + i});
    check(kern::crc32c_batch(items.data(), int(items.size()), reinterpret_cast<void*>(ws), as_stream(stream), cus),
          "crc32c_batch");
  }, py::arg("buffers"), py::arg("out"), py::arg("workspace"), py::arg("stream") = 0, py::arg("cus") = 0);
  m.def("fp8_pack", [](uint64_t bf16, int64_t n, uint64_t fp8, uint64_t scales, int block, uint64_t stream) {
    check(kern::fp8_pack(reinterpret_cast<const uint16_t*>(bf16), n, reinterpret_cast<uint8_t*>(fp8),
                         reinterpret_cast<float*>(scales), block, as_stream(stream)),
          "fp8_pack");
  }, py::arg("bf16"), py::arg("n"), py::arg("fp8"), py::arg("scales"), py::arg("block") = 128, py::arg("stream") = 0);
  m.def("fp8_unpack", [](uint64_t fp8, uint64_t scales, int64_t n, uint64_t bf16, int block, uint64_t stream) {
    check(kern::fp8_unpack(reinterpret_cast<const uint8_t*>(fp8), reinterpret_cast<const float*>(scales), n,
                           reinterpret_cast<uint16_t*>(bf16), block, as_stream(stream)),
          "fp8_unpack");
  }, py::arg("fp8"), py::arg("scales"), py::arg("n"), py::arg("bf16"), py::arg("block") = 128, py::arg("stream") = 0);
  m.def("fp8_pack_chunks", [](uint64_t src, int64_t src_bytes, int64_t src_chunk, int block, uint64_t dst,
                              uint64_t stream) {
    check(kern::fp8_pack_chunks(reinterpret_cast<const void*>(src), src_bytes, src_chunk, block,
                                reinterpret_cast<void*>(dst), as_stream(stream)),
          "fp8_pack_chunks");
  }, py::arg("src"), py::arg("src_bytes"), py::arg("src_chunk"), py::arg("block"), py::arg("dst"),
        py::arg("stream") = 0);
  m.def("fp8_verify_unpack_async", [](uint64_t packed, int64_t src_bytes, int64_t src_chunk, int block,
                                      uint64_t out, uint64_t crc_out_dev, uint64_t ws, uint64_t stream, int cus) {
    check(kern::fp8_verify_unpack(reinterpret_cast<const void*>(packed), src_bytes, src_chunk, block,
                                  reinterpret_cast<uint16_t*>(out), reinterpret_cast<uint32_t*>(crc_out_dev),
                                  reinterpret_cast<void*>(ws), as_stream(stream), cus),
          "fp8_verify_unpack");
  }, py::arg("packed"), py::arg("src_bytes"), py::arg("src_chunk"), py::arg("block"), py::arg("out"),
     py::arg("crc_out"), py::arg("ws"), py::arg("stream") = 0, py::arg("cus") = 0);
  // Fused verify + unpack (synchronous): writes the bf16 layer to `out`, returns
  // the CRC32C of every packed chunk.
  m.def("fp8_verify_unpack", [](uint64_t packed, int64_t src_bytes, int64_t src_chunk, int block, uint64_t out,
                                uint64_t stream, int cus) {
    py::gil_scoped_release nogil;
    const int64_t pbytes = fp8::packed_size(src_bytes, src_chunk, block);
    const int64_t pchunk = fp8::packed_chunk(src_chunk, block);
    const size_t n = size_t((pbytes + pchunk - 1) / pchunk);
    void* ws = nullptr;
    uint32_t *host = nullptr, *dev = nullptr;
    const size_t wsb = kern::crc32c_workspace_bytes(pbytes, pchunk);
    check(hipMalloc(&ws, wsb), "hipMalloc");
    check(hipMemset(ws, 0, wsb), "hipMemset");
    check(hipHostMalloc(reinterpret_cast<void**>(&host), std::max<size_t>(n, 1) * 4, hipHostMallocMapped),
          "hipHostMalloc");
    check(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev), host, 0), "hipHostGetDevicePointer");
    hipError_t e = kern::fp8_verify_unpack(reinterpret_cast<const void*>(packed), src_bytes, src_chunk, block,
                                           reinterpret_cast<uint16_t*>(out), dev, ws, as_stream(stream), cus);
    if (e == hipSuccess) e = hipStreamSynchronize(as_stream(stream));
    std::vector<uint32_t> crc(host, host + n);
    (void)hipFree(ws);
    (void)hipHostFree(host);
    check(e, "fp8_verify_unpack");
    return crc;
  }, py::arg("packed"), py::arg("src_bytes"), py::arg("src_chunk"), py::arg("block"), py::arg("out"),
        py::arg("stream") = 0, py::arg("cus") = 0);
  // Batched fused verify + unpack of independent packed chunks
  // [(packed_ptr, src_len, out_ptr), ...]: the engine's launch for the chunks
  // one P2P group or staging batch landed. _async writes CRCs to crc_out[i].
  auto fused_items = [](const std::vector<std::tuple<uint64_t, int64_t, uint64_t>>& items, uint32_t* crc) {
    if (items.size() > size_t(kern::kCrcBatchMax)) throw std::invalid_argument("too many chunks for one batch");
    std::vector<kern::FusedItem> v;
    for (size_t i = 0; i < items.size(); ++i)
      v.push_back(kern::FusedItem{reinterpret_cast<const void*>(std::get<0>(items[i])), std::get<1>(items[i]),
                                  reinterpret_cast<uint16_t*>(std::get<2>(items[i])), crc + i});
    return v;
  };
  m.def("fp8_verify_unpack_batch_async", [fused_items](const std::vector<std::tuple<uint64_t, int64_t, uint64_t>>& items,
                                                       int block, uint64_t crc_out_dev, uint64_t ws, uint64_t stream,
                                                       int cus) {
    auto v = fused_items(items, reinterpret_cast<uint32_t*>(crc_out_dev));
    check(kern::fp8_verify_unpack_batch(v.data(), int(v.size()), block, reinterpret_cast<void*>(ws), as_stream(stream),
                                        cus),
          "fp8_verify_unpack_batch");
  }, py::arg("items"), py::arg("block"), py::arg("crc_out"), py::arg("ws"), py::arg("stream") = 0, py::arg("cus") = 0);
  m.def("fp8_verify_unpack_batch", [fused_items](const std::vector<std::tuple<uint64_t, int64_t, uint64_t>>& items,
                                                 int block, uint64_t stream, int cus) {
    py::gil_scoped_release nogil;
    void* ws = nullptr;
    uint32_t *host = nullptr, *dev = nullptr;
    check(hipMalloc(&ws, kern::crc32c_batch_workspace_bytes()), "hipMalloc");
    check(hipMemset(ws, 0, kern::crc32c_batch_workspace_bytes()), "hipMemset");
    check(hipHostMalloc(reinterpret_cast<void**>(&host), std::max<size_t>(items.size(), 1) * 4, hipHostMallocMapped),
          "hipHostMalloc");
    check(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev), host, 0), "hipHostGetDevicePointer");
    hipError_t e = hipSuccess;
    try {
      auto v = fused_items(items, dev);
      e = kern::fp8_verify_unpack_batch(v.data(), int(v.size()), block, ws, as_stream(stream), cus);
    } catch (...) {
      (void)hipFree(ws);
      (void)hipHostFree(host);
      throw;
    }
    if (e == hipSuccess) e = hipStreamSynchronize(as_stream(stream));
    std::vector<uint32_t> crc(host, host + items.size());
    (void)hipFree(ws);
    (void)hipHostFree(host);
    check(e, "fp8_verify_unpack_batch");
    return crc;
  }, py::arg("items"), py::arg("block") = 128, py::arg("stream") = 0, py::arg("cus") = 0);

  // ---- RCCL path on one GPU: a one-rank communicator driven through the same
  // Backend::group / crc calls the planned engine issues. `rounds` groups of
  // {send chunk k to self, recv into dst chunk k}, then an in-place broadcast
  // from rank 0; returns (src CRCs, dst CRCs after P2P, CRCs after broadcast).
  m.def("rccl_selftest", [](int device, int64_t bytes, int64_t chunk) {
    py::gil_scoped_release nogil;
    if (bytes <= 0 || chunk <= 0 || chunk % 16) throw std::invalid_argument("bytes > 0, chunk % 16 == 0");
    HipBackendConfig hc;
    hc.device = device;
    hc.max_chunk_bytes = bytes;
    hc.self_comm = true;
    auto be = make_hip_backend(hc);
    be->init_thread();
    uint8_t* src = be->alloc(bytes);
    uint8_t* dst = be->alloc(bytes);
    check(kern::fill_random(src, bytes, 0x5e1f, nullptr), "fill_random");
    check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    be->zero_sync(dst, bytes);
    Ev last = 0;
    for (int64_t off = 0; off < bytes; off += chunk) {
      const int64_t n = std::min(chunk, bytes - off);
      std::vector<XOp> ops{XOp{true, 0, src + off, n}, XOp{false, 0, dst + off, n}};
      std::vector<Ev> waits;
      if (last) waits.push_back(last);
      last = be->group(ops, waits);
    }
    auto wait = [&](Ev e) {
      int q;
      while ((q = be->query(e)) == 0) std::this_thread::yield();
      if (q < 0) throw std::runtime_error("rccl_selftest: " + be->async_error());
    };
    wait(last);
    std::vector<uint32_t> a = crc_chunks_sync(reinterpret_cast<uint64_t>(src), bytes, chunk, 0);
    std::vector<uint32_t> b = crc_chunks_sync(reinterpret_cast<uint64_t>(dst), bytes, chunk, 0);
    XOp bc{false, 0, dst, bytes};
    bc.bcast = true;
    Ev e = be->group({bc}, {last});
    wait(e);
    std::vector<uint32_t> c = crc_chunks_sync(reinterpret_cast<uint64_t>(dst), bytes, chunk, 0);
    std::string err = be->async_error();
    be->free(src);
    be->free(dst);
    be->destroy(false);
    if (!err.empty()) throw std::runtime_error("rccl_selftest: " + err);
    return std::make_tuple(a, b, c);
  }, py::arg("device"), py::arg("bytes"), py::arg("chunk"));

  // ---- RCCL engine = planned engine on the HIP backend
  m.def("nccl_unique_id", [](int count) { return py::bytes(nccl_unique_id(count)); }, py::arg("count") = 1);
  m.def("gpu_engine", [](const PlannedConfig& cfg, int device, py::bytes uid) {
    HipBackendConfig hc;
    hc.device = device;
    hc.rank = cfg.rank;
    hc.world = cfg.world;
    hc.nccl_uid = std::string(uid);
    hc.max_chunk_bytes = cfg.chunk_bytes;
    hc.reserve_cus = cfg.reserve_cus >= 0 ? cfg.reserve_cus : (cfg.world > 1 ? 32 : 0);
    // with peers the verify owns the last 32 CUs (128 with the fused unpack) and
    // RCCL the rest (hip_backend.h verify_cus)
    hc.verify_cus = cfg.verify_cus >= 0 ? cfg.verify_cus : (cfg.world > 1 ? (cfg.unpack_store ? 128 : 32) : 0);
    hc.nccl_min_ctas = cfg.nccl_min_ctas;
    hc.nccl_max_ctas = cfg.nccl_max_ctas;
    hc.nccl_register = cfg.nccl_register;
    hc.lanes = resolve_lanes(cfg);
    hc.hosts = cfg.hosts;
    hc.host_lane_classes = cfg.host_lane_classes;
    if (cfg.comm_init != "parallel" && cfg.comm_init != "split")
      throw std::runtime_error("comm_init must be parallel or split, not " + cfg.comm_init);
    hc.parallel_init = cfg.comm_init == "parallel";
    py::gil_scoped_release nogil;
    return std::make_shared<PlannedEngine>(cfg, make_hip_backend(hc));
  }, py::arg("cfg"), py::arg("device") = 0, py::arg("nccl_uid") = py::bytes(""));
}
