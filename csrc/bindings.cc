// pybind11 module `_core`: the Python face of the native runtime. Python only
// wires things together (CLI, config, bench); every state machine, transport,
// scheduler and data engine runs in C++ threads with the GIL released.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "core/crc32c.h"
#include "core/fp8.h"
#include "core/log.h"
#include "core/ratelimit.h"
#include "core/trace.h"
#include "core/vclock.h"
#include "core/wire.h"
#include "engine/engine.h"
#include "engine/planned_engine.h"
#include "gpu/gpu_api.h"
#include "roles/plan_cache.h"
#include "roles/node.h"
#include "sched/lp.h"
#include "sched/maxflow.h"
#include "store/store.h"
#include "transport/transport.h"

namespace py = pybind11;
using namespace dissem;

namespace {

// Barrier for the threads of an in-process simulation (a threading.Barrier
// would hold a clock-counted thread busy and stop model time).
class VBarrier {
 public:
  explicit VBarrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> lk(mu_);
    const uint64_t gen = gen_;
    if (++count_ >= n_) {
      count_ = 0;
      ++gen_;
      lk.unlock();
      cv_.notify_all();
      return;
    }
    cv_.wait(lk, [&] { return gen_ != gen; });
  }

 private:
  std::mutex mu_;
  CondVar cv_;
  int n_, count_ = 0;
  uint64_t gen_ = 0;
};

std::shared_ptr<HostBuffer> buffer_from_py(const py::object& obj) {
  py::buffer buf = py::reinterpret_borrow<py::buffer>(obj);
  py::buffer_info info = buf.request();
  int64_t n = int64_t(info.size) * int64_t(info.itemsize);
  auto hb = HostBuffer::alloc(n, false);
  if (n) memcpy(hb->ptr, info.ptr, size_t(n));
  return hb;
}

py::bytes host_bytes(const std::shared_ptr<HostBuffer>& b, int64_t off, int64_t n) {
  if (!b) return py::bytes("");
  if (n < 0) n = b->size - off;
  return py::bytes(reinterpret_cast<const char*>(b->ptr + off), size_t(n));
}

Assignment assignment_from(const py::dict& d) {
  Assignment a;
  for (auto item : d) {
    NodeID n = item.first.cast<NodeID>();
    LayerIDs ids;
    for (auto l : item.second) ids[l.cast<LayerID>()] = LayerMeta{};
    a[n] = ids;
  }
  return a;
}

}  // namespace

PYBIND11_MODULE(_core, m) {
  m.doc() = "MI355X-native layer dissemination runtime (C++/HIP core)";

  // ---- logging
  m.def("set_log_level", &log::set_level);
  // The process-wide leader plan cache (roles/plan_cache.h): tests that count cache hits start empty.
  m.def("plan_cache_clear", [] { PlanCache::instance().clear(); });
  m.def("log_level", [] { return int(log::level()); });
  m.def("set_log_file", &log::set_file);
  // ---- roctx (rocprofv3 --marker-trace)
  m.def("trace_available", &trace::available);
  m.def("trace_mark", [](const std::string& s) { trace::mark(s.c_str()); });
  m.def("trace_push", [](const std::string& s) { trace::push(s.c_str()); });
  m.def("trace_pop", &trace::pop);

  // ---- enums
  py::enum_<Location>(m, "Location")
      .value("Inmem", Location::Inmem)
      .value("Disk", Location::Disk)
      .value("Client", Location::Client)
      .value("Device", Location::Device);
  py::enum_<SourceType>(m, "SourceType")
      .value("Client", SourceType::Client)
      .value("Disk", SourceType::Disk)
      .value("Mem", SourceType::Mem)
      .value("Device", SourceType::Device);
  py::enum_<MsgType>(m, "MsgType")
      .value("Announce", MsgType::Announce)
      .value("Ack", MsgType::Ack)
      .value("Layer", MsgType::Layer)
      .value("Retransmit", MsgType::Retransmit)
      .value("FlowRetransmit", MsgType::FlowRetransmit)
      .value("ClientReq", MsgType::ClientReq)
      .value("Startup", MsgType::Startup)
      .value("Simple", MsgType::Simple)
      .value("Transport", MsgType::Transport)
      .value("Nack", MsgType::Nack)
      .value("Bcast", MsgType::Bcast)
      .value("Landed", MsgType::Landed)
      .value("XferBatch", MsgType::XferBatch);
  m.attr("CLIENT_ID") = py::int_(kClientID);

  py::class_<LayerMeta>(m, "LayerMeta")
      .def(py::init<>())
      .def(py::init([](Location loc, int64_t rate, SourceType st, int64_t size) {
             return LayerMeta{loc, rate, st, size};
           }),
           py::arg("location") = Location::Inmem, py::arg("limit_rate") = 0,
           py::arg("source_type") = SourceType::Client, py::arg("size") = 0)
      .def_readwrite("location", &LayerMeta::location)
      .def_readwrite("limit_rate", &LayerMeta::limit_rate)
      .def_readwrite("source_type", &LayerMeta::source_type)
      .def_readwrite("size", &LayerMeta::size)
      .def("__eq__", [](const LayerMeta& a, const LayerMeta& b) {
        return a.location == b.location && a.limit_rate == b.limit_rate && a.source_type == b.source_type;
      })
      .def("__repr__", [](const LayerMeta& x) {
        return "LayerMeta(" + std::string(location_name(x.location)) + ", rate=" + std::to_string(x.limit_rate) +
               ", src=" + std::to_string(int(x.source_type)) + ", size=" + std::to_string(x.size) + ")";
      });

  // ---- messages / codec
  py::class_<XferJob>(m, "XferJob")
      .def(py::init<>())
      .def_readwrite("seq", &XferJob::seq)
      .def_readwrite("src", &XferJob::src)
      .def_readwrite("dst", &XferJob::dst)
      .def_readwrite("layer", &XferJob::layer)
      .def_readwrite("offset", &XferJob::offset)
      .def_readwrite("size", &XferJob::size)
      .def_readwrite("total", &XferJob::total)
      .def_readwrite("chunk_bytes", &XferJob::chunk_bytes)
      .def_readwrite("crc", &XferJob::crc)
      .def_readwrite("rate", &XferJob::rate);
  py::class_<Message, MessagePtr>(m, "Message")
      .def(py::init<>())
      .def_readwrite("type", &Message::type)
      .def_readwrite("src", &Message::src)
      .def_readwrite("src_str", &Message::src_str)
      .def_readwrite("epoch", &Message::epoch)
      .def_readwrite("layers", &Message::layers)
      .def_readwrite("layer", &Message::layer)
      .def_readwrite("dest", &Message::dest)
      .def_readwrite("data_size", &Message::data_size)
      .def_readwrite("offset", &Message::offset)
      .def_readwrite("rate", &Message::rate)
      .def_readwrite("total_size", &Message::total_size)
      .def_readwrite("location", &Message::location)
      .def_readwrite("partial", &Message::partial)
      .def_readwrite("save_disk", &Message::save_disk)
      .def_readwrite("chunk_bytes", &Message::chunk_bytes)
      .def_readwrite("crc", &Message::crc)
      .def_readwrite("seq", &Message::seq)
      .def_readwrite("batch", &Message::batch)
      .def_readwrite("order", &Message::order)
      .def_readwrite("jobs", &Message::jobs)
      .def_readwrite("peers", &Message::peers)
      .def_readwrite("src_addr", &Message::src_addr)
      .def_readwrite("payload_str", &Message::payload_str)
      .def("payload_bytes", [](const Message& x) { return host_bytes(x.data, x.data_off, x.data_size); })
      .def("__str__", &Message::str)
      .def("__repr__", [](const Message& x) { return std::string("<Message ") + msg_type_name(x.type) + " " + x.str() + ">"; });
  m.def("simple_msg", [](const std::string& src, const std::string& payload) {
    auto x = std::make_shared<Message>();
    x->type = MsgType::Simple;
    x->src_addr = src;
    x->payload_str = payload;
    return x;
  });
  m.def("encode_envelope", [](const Message& x) { return py::bytes(encode_envelope(x)); });
  m.def("decode_envelope", [](const std::string& s) { return decode_envelope(Json::parse(s)); });
  m.def("decode_envelope_text", [](const std::string& s) { return decode_envelope_text(s.data(), s.size()); },
        "the transport's decoder (transfer batches take the fast path)");
  m.def("json_roundtrip", [](const std::string& s) { return Json::parse(s).dump(); });
  m.def("json_parse_prefix", [](const std::string& s) {
    Json out;
    size_t n = Json::parse_prefix(s.data(), s.size(), out);
    return py::make_tuple(n, n ? out.dump() : std::string());
  });

  // ---- layers
  py::class_<LayerSrc>(m, "LayerSrc")
      .def(py::init<>())
      .def_static("inmem", [](py::object data_or_size, int64_t rate, SourceType st) {
        LayerSrc s;
        if (py::isinstance<py::int_>(data_or_size)) {
          int64_t n = data_or_size.cast<int64_t>();
          s.host = HostBuffer::alloc(n < 0 ? 0 : n, true);  // cmd/config.go:159-171 (negative clamps to 0)
        } else {
          s.host = buffer_from_py(data_or_size);
        }
        s.data_size = s.host->size;
        s.meta = LayerMeta{Location::Inmem, rate, st, s.data_size};
        return s;
      }, py::arg("data_or_size"), py::arg("limit_rate") = 0, py::arg("source_type") = SourceType::Mem)
      .def_static("disk", [](const std::string& path, int64_t size, int64_t rate, SourceType st) {
        LayerSrc s;
        s.path = path;
        s.data_size = size;
        s.meta = LayerMeta{Location::Disk, rate, st, size};
        return s;
      }, py::arg("path"), py::arg("size"), py::arg("limit_rate") = 0, py::arg("source_type") = SourceType::Disk)
      .def_static("client", [](int64_t size, int64_t rate) {
        LayerSrc s;
        s.data_size = size;
        s.meta = LayerMeta{Location::Client, rate, SourceType::Client, size};
        return s;
      }, py::arg("size"), py::arg("limit_rate") = 0)
      .def_readwrite("path", &LayerSrc::path)
      .def_readwrite("data_size", &LayerSrc::data_size)
      .def_readwrite("offset", &LayerSrc::offset)
      .def_readwrite("meta", &LayerSrc::meta)
      .def_readwrite("ranges", &LayerSrc::ranges)
      .def_property_readonly("has_host", [](const LayerSrc& s) { return bool(s.host); })
      .def_property_readonly("dev_ptr", [](const LayerSrc& s) { return reinterpret_cast<uintptr_t>(s.dev); })
      .def("host_bytes", [](const LayerSrc& s) { return host_bytes(s.host, 0, s.host ? s.host->size : 0); });

  // ---- transports
  py::class_<Transport, std::shared_ptr<Transport>>(m, "Transport")
      .def("send", [](Transport& t, NodeID dest, const Message& msg) {
        py::gil_scoped_release nogil;
        t.send(dest, msg);
      })
      .def("broadcast", [](Transport& t, const Message& msg) {
        py::gil_scoped_release nogil;
        t.broadcast(msg);
      })
      .def("deliver", [](Transport& t, double timeout) -> py::object {
        std::optional<MessagePtr> r;
        {
          py::gil_scoped_release nogil;
          r = t.deliver().pop_for(timeout);
        }
        if (!r) return py::none();
        return py::cast(*r);
      }, py::arg("timeout") = 1.0)
      .def("register_pipe", &Transport::register_pipe)
      .def("address", &Transport::address)
      .def("set_registry", &Transport::set_registry)
      .def("set_max_envelope", &Transport::set_max_envelope, "largest control envelope a peer may send (bytes)")
      .def("set_max_payload", &Transport::set_max_payload, "largest layer message DataSize / TotalSize (bytes)")
      .def("add_peer", &Transport::add_peer)
      .def("registry", &Transport::registry)
      .def_property_readonly("bytes_sent", [](const Transport& t) { return t.bytes_sent.load(); })
      .def_property_readonly("bytes_received", [](const Transport& t) { return t.bytes_received.load(); })
      .def("close", [](Transport& t) {
        py::gil_scoped_release nogil;
        t.close();
      });
  m.def("inproc_transport", &make_inproc_transport, py::arg("addr"), py::arg("registry") = AddrRegistry{});
  m.def("tcp_transport", [](const std::string& addr, const AddrRegistry& reg, bool is_client) {
    py::gil_scoped_release nogil;
    return make_tcp_transport(addr, reg, is_client);
  }, py::arg("addr"), py::arg("registry") = AddrRegistry{}, py::arg("is_client") = false);

  // ---- engines
  py::class_<DataEngine, std::shared_ptr<DataEngine>>(m, "DataEngine")
      .def_property_readonly("name", &DataEngine::name)
      .def_property_readonly("target", &DataEngine::target)
      .def("shutdown", [](DataEngine& e) {
        py::gil_scoped_release nogil;
        e.shutdown();
      });
  m.def("host_engine", &make_host_engine, py::arg("link_rate") = std::map<NodeID, int64_t>{});

  py::class_<CrcManifest>(m, "CrcManifest")
      .def(py::init<>())
      .def(py::init([](int64_t cb, std::vector<uint32_t> crc) { return CrcManifest{cb, std::move(crc)}; }))
      .def_readwrite("chunk_bytes", &CrcManifest::chunk_bytes)
      .def_readwrite("crc", &CrcManifest::crc);
  py::class_<PlannedConfig>(m, "PlannedConfig")
      .def(py::init<>())
      .def_readwrite("rank", &PlannedConfig::rank)
      .def_readwrite("world", &PlannedConfig::world)
      .def_readwrite("rank_nodes", &PlannedConfig::rank_nodes)
      .def_readwrite("chunk_bytes", &PlannedConfig::chunk_bytes)
      .def_readwrite("verify", &PlannedConfig::verify)
      .def_readwrite("poison", &PlannedConfig::poison)
      .def_readwrite("max_inflight_groups", &PlannedConfig::max_inflight_groups)
      .def_readwrite("group_peers", &PlannedConfig::group_peers)
      .def_readwrite("disk_o_direct", &PlannedConfig::disk_o_direct)
      .def_readwrite("disk_readers", &PlannedConfig::disk_readers)
      .def_readwrite("disk_ring", &PlannedConfig::disk_ring)
      .def_readwrite("pack", &PlannedConfig::pack)
      .def_readwrite("pack_block", &PlannedConfig::pack_block)
      .def_readwrite("max_retries", &PlannedConfig::max_retries)
      .def_readwrite("inject_corrupt", &PlannedConfig::inject_corrupt)
      .def_readwrite("inject_seed", &PlannedConfig::inject_seed)
      .def_readwrite("group_timeout_s", &PlannedConfig::group_timeout_s)
      .def_readwrite("reserve_cus", &PlannedConfig::reserve_cus)
      .def_readwrite("verify_cus", &PlannedConfig::verify_cus)
      .def_readwrite("suspect_s", &PlannedConfig::suspect_s)
      .def_readwrite("inject_die_after_groups", &PlannedConfig::inject_die_after_groups)
      .def_readwrite("nccl_min_ctas", &PlannedConfig::nccl_min_ctas)
      .def_readwrite("nccl_max_ctas", &PlannedConfig::nccl_max_ctas)
      .def_readwrite("nccl_register", &PlannedConfig::nccl_register)
      .def_readwrite("lanes", &PlannedConfig::lanes)
      .def_readwrite("hosts", &PlannedConfig::hosts)
      .def_readwrite("host_lane_classes", &PlannedConfig::host_lane_classes)
      .def_readwrite("unpack_store", &PlannedConfig::unpack_store)
      .def_readwrite("link_rate", &PlannedConfig::link_rate)
      .def_readwrite("comm_init", &PlannedConfig::comm_init)
      .def_readwrite("node_disk_rate", &PlannedConfig::node_disk_rate)
      .def_readwrite("node_disk_key", &PlannedConfig::node_disk_key);
  m.def("resolve_lanes", [](int world, int lanes, int hosts, int classes) {
    PlannedConfig c;
    c.world = world;
    c.lanes = lanes;
    c.hosts = hosts;
    c.host_lane_classes = classes;
    return resolve_lanes(c);
  }, py::arg("world"), py::arg("lanes") = 0, py::arg("hosts") = 1, py::arg("classes") = 0);
  m.def("lane_of", [](int src, int dst, int world, int lanes, int hosts, int classes) {
    return lane_of_hosts(src, dst, world, lanes, hosts, classes);
  }, py::arg("src"), py::arg("dst"), py::arg("world"), py::arg("lanes"), py::arg("hosts") = 1,
     py::arg("classes") = 0);
  py::class_<PlannedStats>(m, "PlannedStats")
      .def_readonly("bytes_sent", &PlannedStats::bytes_sent)
      .def_readonly("bytes_recv", &PlannedStats::bytes_recv)
      .def_readonly("bytes_staged", &PlannedStats::bytes_staged)
      .def_readonly("bytes_verified", &PlannedStats::bytes_verified)
      .def_readonly("groups", &PlannedStats::groups)
      .def_readonly("pieces", &PlannedStats::pieces)
      .def_readonly("verify_failures", &PlannedStats::verify_failures)
      .def_readonly("unverified_pieces", &PlannedStats::unverified_pieces)
      .def_readonly("nacks", &PlannedStats::nacks)
      .def_readonly("injected", &PlannedStats::injected)
      .def_readonly("issue_ms", &PlannedStats::issue_ms)
      .def_readonly("verify_busy_ms", &PlannedStats::verify_busy_ms)
      .def_readonly("peer_sent", &PlannedStats::peer_sent)
      .def_readonly("peer_recv", &PlannedStats::peer_recv)
      .def_readonly("group_us_hist", &PlannedStats::group_us_hist)
      .def_readonly("land_us_hist", &PlannedStats::land_us_hist)
      .def_readonly("suspects", &PlannedStats::suspects)
      .def_readonly("shrinks", &PlannedStats::shrinks)
      .def_readonly("aborted_pieces", &PlannedStats::aborted_pieces)
      .def_readonly("peer_busy_ms", &PlannedStats::peer_busy_ms)
      .def_readonly("peer_send_busy_ms", &PlannedStats::peer_send_busy_ms)
      .def_readonly("peer_recv_busy_ms", &PlannedStats::peer_recv_busy_ms)
      .def_readonly("verify_calls", &PlannedStats::verify_calls)
      .def_readonly("verify_chunks", &PlannedStats::verify_chunks)
      .def_readonly("lane_busy_ms", &PlannedStats::lane_busy_ms)
      .def_readonly("lanes", &PlannedStats::lanes)
      .def_readonly("comm_init_ms", &PlannedStats::comm_init_ms)
      .def_readonly("comm_connect_ms", &PlannedStats::comm_connect_ms)
      .def_readonly("lane_init_ms", &PlannedStats::lane_init_ms)
      .def_readonly("lane_connect_ms", &PlannedStats::lane_connect_ms)
      .def_readonly("comm_reform_ms", &PlannedStats::comm_reform_ms)
      .def_readonly("paced", &PlannedStats::paced)
      .def_readonly("disk_wait_ms", &PlannedStats::disk_wait_ms)
      .def_readonly("disk_direct_bytes", &PlannedStats::disk_direct_bytes)
      .def_readonly("scratch_landings", &PlannedStats::scratch_landings)
      .def_readonly("scratch_buffers", &PlannedStats::scratch_buffers)
      .def_readonly("disk_buffered_bytes", &PlannedStats::disk_buffered_bytes)
      .def_readonly("order_violations", &PlannedStats::order_violations);
  py::class_<PlannedEngine, DataEngine, std::shared_ptr<PlannedEngine>>(m, "PlannedEngine")
      .def("provision", [](PlannedEngine& e, LayerID l, int64_t n) {
        return reinterpret_cast<uint64_t>(e.provision(l, n));
      })
      .def("slot_size", &PlannedEngine::slot_size)
      .def_property_readonly("chunk_grid", &PlannedEngine::chunk_bytes)
      .def("device_ptr", [](PlannedEngine& e, LayerID l) { return reinterpret_cast<uint64_t>(e.device_ptr(l)); })
      .def("unpacked_ptr", [](PlannedEngine& e, LayerID l) { return reinterpret_cast<uint64_t>(e.unpacked_ptr(l)); })
      .def("set_manifest", &PlannedEngine::set_manifest)
      .def("manifest", &PlannedEngine::manifest)
      .def("set_source_packed", &PlannedEngine::set_source_packed)
      .def("set_seeded", &PlannedEngine::set_seeded)
      .def("resident_chunks", &PlannedEngine::resident_chunks)
      .def("reset_session", [](PlannedEngine& e) {
        py::gil_scoped_release nogil;
        e.reset_session();
      })
      .def("quiesce", [](PlannedEngine& e) {
        py::gil_scoped_release nogil;
        e.quiesce();
      })
      .def("stats", &PlannedEngine::stats)
      .def("probe", [](PlannedEngine& e, const std::vector<std::tuple<int, bool, int64_t>>& ops, double timeout_s) {
        std::vector<ProbeOp> in;
        for (auto& t : ops) {
          ProbeOp o;
          o.peer = std::get<0>(t);
          o.send = std::get<1>(t);
          o.bytes = std::get<2>(t);
          in.push_back(o);
        }
        std::vector<ProbeOp> out;
        {
          py::gil_scoped_release nogil;
          out = e.probe(in, timeout_s);
        }
        py::list res;
        for (auto& o : out) {
          py::dict d;
          d["peer"] = o.peer;
          d["send"] = o.send;
          d["bytes"] = o.bytes;
          d["done"] = o.done;
          d["ms"] = o.ms;
          d["lane"] = o.lane;
          res.append(d);
        }
        return res;
      }, py::arg("ops"), py::arg("timeout_s") = 30.0)
      .def("error", &PlannedEngine::error)
      .def_property_readonly("backend", [](PlannedEngine& e) { return e.backend()->name(); });
  // Simulated fabric (CPU): host "device" memory, RCCL P2P matching semantics between
  // in-process ranks that share `comm_key`.
  m.def("sim_engine", [](const PlannedConfig& cfg, const std::string& comm_key) {
    return std::make_shared<PlannedEngine>(cfg, make_sim_backend(comm_key, cfg.rank, cfg.world, resolve_lanes(cfg)));
  });
  py::class_<SimTiming>(m, "SimTiming")
      .def(py::init<>())
      .def_readwrite("link_bps", &SimTiming::link_bps)
      .def_readwrite("link", &SimTiming::link)
      .def_readwrite("stage_bps", &SimTiming::stage_bps)
      .def_readwrite("copy_bytes", &SimTiming::copy_bytes)
      .def_readwrite("p2p_rounds", &SimTiming::p2p_rounds)
      .def_readwrite("host", &SimTiming::host)
      .def_readwrite("nic_bps", &SimTiming::nic_bps)
      .def_readwrite("wait_s", &SimTiming::wait_s)
      .def_readwrite("recv_delay_s", &SimTiming::recv_delay_s)
      .def_readwrite("serialize_lanes", &SimTiming::serialize_lanes)
      .def_readwrite("trace", &SimTiming::trace)
      .def_readwrite("verify_bps", &SimTiming::verify_bps)
      .def_readwrite("verify_launch_s", &SimTiming::verify_launch_s);
  m.def("sim_set_timing", &sim_set_timing, py::arg("comm_key"), py::arg("timing"));
  // Virtual clock (core/vclock.h): the simulator in model time. Python threads
  // that drive a session's ranks are counted by the clock between adopt() and
  // release() (reserve first, from the thread that starts them).
  m.def("file_cache_drop", [](const std::string& p) {
    py::gil_scoped_release nogil;
    return file_cache_drop(p);
  }, "write back and evict a file's page-cache pages; returns the fraction still resident");
  m.def("file_cache_resident", [](const std::string& p) {
    py::gil_scoped_release nogil;
    return file_cache_resident(p);
  }, "fraction of a file's pages in the page cache (mincore)");
  m.def("vclock_enable", [](bool on) { vclock::enable(on); });
  m.def("vclock_enabled", &vclock::enabled);
  m.def("vclock_now", &vclock::now, "seconds: model time when the virtual clock is on, else the steady clock");
  m.def("vclock_reserve", &vclock::reserve, py::arg("n"));
  m.def("vclock_adopt", [] { vclock::adopt("python"); });
  m.def("vclock_release", &vclock::release);
  m.def("vclock_sleep", [](double s) {
    py::gil_scoped_release nogil;
    vclock::sleep_for(s);
  });
  m.def("vclock_stats", [] {
    auto st = vclock::stats();
    py::dict d;
    d["t"] = st.t;
    d["busy"] = st.busy;
    d["blocked"] = st.blocked;
    d["timers"] = st.timers;
    d["advances"] = st.advances;
    return d;
  });
  m.def("vclock_describe", &vclock::describe);
  py::class_<VBarrier, std::shared_ptr<VBarrier>>(m, "VBarrier", "a thread barrier that waits in model time")
      .def(py::init<int>())
      .def("wait", [](VBarrier& b) {
        py::gil_scoped_release nogil;
        b.wait();
      });
  m.def("sim_fabric_bytes", [](const std::string& key) { return sim_fabric_stats(key).bytes; });
  m.def("sim_fabric_trace", [](const std::string& key) {
    auto st = sim_fabric_stats(key);
    return py::make_tuple(st.transfers, st.stages);
  }, "(transfers [(src, dst, start_s, end_s, bytes)], stages [(rank, start_s, end_s, bytes)]) with SimTiming.trace");
  m.def("sim_fabric_clear_trace", [](const std::string& key) { sim_clear_trace(key); });
  m.def("sim_read", [](uint64_t ptr, int64_t n) {
    return py::bytes(reinterpret_cast<const char*>(ptr), size_t(n));
  });
  m.def("sim_write", [](uint64_t ptr, py::bytes data) {
    std::string s(data);
    memcpy(reinterpret_cast<void*>(ptr), s.data(), s.size());
  });
  m.def("host_crc32c_chunks", [](uint64_t ptr, int64_t n, int64_t chunk) {
    std::vector<uint32_t> out;
    for (int64_t off = 0; off < n; off += chunk)
      out.push_back(crc32c(reinterpret_cast<const void*>(ptr + uint64_t(off)), size_t(std::min(chunk, n - off))));
    return out;
  });
  // token bucket (core/ratelimit.h): pace `total` bytes at `rate` B/s; returns
  // (seconds elapsed, piece sizes) - unit-test hook
  // The pacing schedule of `total` bytes on a virtual clock: (seconds the
  // bucket made the caller wait, piece sizes) - exact, whatever the host load.
  m.def("token_bucket_pace", [](int64_t total, int64_t rate, int64_t burst) {
    std::vector<int64_t> pieces;
    BasicTokenBucket<VirtualClock> tb(rate, burst);
    tb.paced(total, [&](int64_t, int64_t n) { pieces.push_back(n); });
    return py::make_tuple(tb.clock().now(), pieces);
  }, py::arg("total"), py::arg("rate"), py::arg("burst") = TokenBucket::kDefaultBurst);
  // fp8 wire/storage format (core/fp8.h), host reference
  m.def("fp8_packed_size", &fp8::packed_size, py::arg("src_bytes"), py::arg("src_chunk"), py::arg("block") = 128);
  m.def("fp8_source_size", &fp8::source_size, py::arg("packed"), py::arg("src_chunk"), py::arg("block") = 128);
  m.def("fp8_pack_layer_host", [](py::bytes src, int64_t src_chunk, int block) {
    std::string s(src);
    std::string out(size_t(fp8::packed_size(int64_t(s.size()), src_chunk, block)), '\0');
    {
      py::gil_scoped_release nogil;
      fp8::pack_layer_host(reinterpret_cast<const uint8_t*>(s.data()), int64_t(s.size()), src_chunk, block,
                           reinterpret_cast<uint8_t*>(out.data()));
    }
    return py::bytes(out);
  }, py::arg("src"), py::arg("src_chunk"), py::arg("block") = 128);
  m.def("fp8_pack_layer_into", [](uint64_t src, int64_t src_bytes, int64_t src_chunk, int block, uint64_t dst) {
    py::gil_scoped_release nogil;
    fp8::pack_layer_host(reinterpret_cast<const uint8_t*>(src), src_bytes, src_chunk, block,
                         reinterpret_cast<uint8_t*>(dst));
  });
  m.def("fp8_unpack_layer_host", [](py::bytes packed, int64_t src_bytes, int64_t src_chunk, int block) {
    std::string s(packed);
    if (int64_t(s.size()) != fp8::packed_size(src_bytes, src_chunk, block))
      throw std::runtime_error("packed buffer size does not match src_bytes");
    std::string out(size_t(src_bytes), '\0');
    {
      py::gil_scoped_release nogil;
      fp8::unpack_layer_host(reinterpret_cast<const uint8_t*>(s.data()), src_bytes, src_chunk, block,
                             reinterpret_cast<uint8_t*>(out.data()));
    }
    return py::bytes(out);
  }, py::arg("packed"), py::arg("src_bytes"), py::arg("src_chunk"), py::arg("block") = 128);

  // ---- roles
  py::class_<NodeConfig>(m, "NodeConfig")
      .def(py::init<>())
      .def_readwrite("id", &NodeConfig::id)
      .def_readwrite("leader", &NodeConfig::leader)
      .def_readwrite("mode", &NodeConfig::mode)
      .def_readwrite("epoch", &NodeConfig::epoch)
      .def_readwrite("seed", &NodeConfig::seed)
      .def_readwrite("owner_policy", &NodeConfig::owner_policy)
      .def_readwrite("pull_window", &NodeConfig::pull_window)
      .def_readwrite("network_bw", &NodeConfig::network_bw)
      .def_readwrite("link_bw", &NodeConfig::link_bw)
      .def_readwrite("stage_bw", &NodeConfig::stage_bw)
      .def_readwrite("hbm_bw", &NodeConfig::hbm_bw)
      .def_readwrite("integer_seconds", &NodeConfig::integer_seconds)
      .def_readwrite("align", &NodeConfig::align)
      .def_readwrite("storage_path", &NodeConfig::storage_path)
      .def_readwrite("relay", &NodeConfig::relay)
      .def_readwrite("collective", &NodeConfig::collective)
      .def_readwrite("pull_job_bytes", &NodeConfig::pull_job_bytes)
      .def_readwrite("range_acks", &NodeConfig::range_acks)
      .def_readwrite("job_timeout_s", &NodeConfig::job_timeout_s)
      .def_readwrite("job_min_rate", &NodeConfig::job_min_rate)
      .def_readwrite("max_redispatch", &NodeConfig::max_redispatch)
      .def_readwrite("link_report", &NodeConfig::link_report)
      .def_readwrite("link_report_in", &NodeConfig::link_report_in)
      .def_readwrite("adapt_links", &NodeConfig::adapt_links)
      .def_readwrite("disk_group", &NodeConfig::disk_group)
      .def_readwrite("disk_group_bw", &NodeConfig::disk_group_bw)
      .def_readwrite("host_share", &NodeConfig::host_share)
      .def_readwrite("host", &NodeConfig::host)
      .def_readwrite("nic_bw", &NodeConfig::nic_bw);
  py::class_<NodeStats>(m, "NodeStats")
      .def_readonly("time_to_deliver_s", &NodeStats::time_to_deliver_s)
      .def_readonly("bytes_planned", &NodeStats::bytes_planned)
      .def_readonly("jobs_dispatched", &NodeStats::jobs_dispatched)
      .def_readonly("layers_received", &NodeStats::layers_received)
      .def_readonly("bytes_received", &NodeStats::bytes_received)
      .def_readonly("flow_T", &NodeStats::flow_T)
      .def_readonly("plan_ms", &NodeStats::plan_ms)
      .def_readonly("plan_cached", &NodeStats::plan_cached)
      .def_readonly("plan_solver", &NodeStats::plan_solver)
      .def_readonly("plan_gap_bytes", &NodeStats::plan_gap_bytes)
      .def_readonly("plan_sched_ms", &NodeStats::plan_sched_ms)
      .def_readonly("plan_dispatch_ms", &NodeStats::plan_dispatch_ms)
      .def_readonly("nacks", &NodeStats::nacks)
      .def_readonly("redispatched", &NodeStats::redispatched)
      .def_readonly("suspects", &NodeStats::suspects)
      .def_readonly("recoveries", &NodeStats::recoveries)
      .def_readonly("dropped", &NodeStats::dropped);
  py::class_<Node, std::shared_ptr<Node>>(m, "Node")
      .def(py::init([](const NodeConfig& cfg, std::shared_ptr<Transport> t, std::shared_ptr<DataEngine> e,
                       const LayersSrc& layers, const py::dict& assignment, bool is_leader) {
             return std::make_shared<Node>(cfg, t, e, layers, assignment_from(assignment), is_leader);
           }),
           py::arg("cfg"), py::arg("transport"), py::arg("engine"), py::arg("layers"),
           py::arg("assignment") = py::dict(), py::arg("is_leader") = false)
      .def("start", &Node::start)
      .def("plan_link_bw", &Node::plan_link_bw)
      .def("stop", [](Node& n) {
        py::gil_scoped_release nogil;
        n.stop();
      })
      .def("announce", [](Node& n) {
        py::gil_scoped_release nogil;
        n.announce();
      })
      .def("wait_ready", [](Node& n, double t) {
        py::gil_scoped_release nogil;
        return n.wait_ready(t);
      }, py::arg("timeout") = 1.0)
      .def("wait_start", [](Node& n, double t) {
        py::gil_scoped_release nogil;
        return n.wait_start(t);
      }, py::arg("timeout") = 1.0)
      .def("assignment", [](Node& n) {
        std::map<NodeID, std::vector<LayerID>> out;
        for (auto& kv : n.assignment())
          for (auto& l : kv.second) out[kv.first].push_back(l.first);
        return out;
      })
      .def("status", &Node::status)
      .def("stats", &Node::stats)
      .def("inventory", [](Node& n) { return n.store().inventory(); })
      .def("layer", [](Node& n, LayerID l) -> py::object {
        LayerSrc s;
        if (!n.store().get(l, &s)) return py::none();
        return py::cast(s);
      })
      .def("add_node", &Node::add_node)
      .def("update_leader", &Node::update_leader)
      .def("next_hop", &Node::next_hop)
      .def_property_readonly("id", &Node::id);
  py::class_<ClientNode, std::shared_ptr<ClientNode>>(m, "ClientNode")
      .def(py::init<NodeID, std::shared_ptr<Transport>, const LayersSrc&>())
      .def("start", &ClientNode::start)
      .def("stop", [](ClientNode& c) {
        py::gil_scoped_release nogil;
        c.stop();
      });

  // ---- scheduler
  py::class_<FlowJob>(m, "FlowJob")
      .def_readonly("sender", &FlowJob::sender)
      .def_readonly("layer", &FlowJob::layer)
      .def_readonly("dest", &FlowJob::dest)
      .def_readonly("size", &FlowJob::size)
      .def_readonly("offset", &FlowJob::offset)
      .def("__repr__", [](const FlowJob& j) {
        return "FlowJob(s" + std::to_string(j.sender) + "->d" + std::to_string(j.dest) + " l" +
               std::to_string(j.layer) + " [" + std::to_string(j.offset) + "+" + std::to_string(j.size) + "])";
      });
  py::class_<FlowPlan>(m, "FlowPlan")
      .def_readonly("T", &FlowPlan::T)
      .def_readonly("required", &FlowPlan::required)
      .def_readonly("max_flow", &FlowPlan::max_flow)
      .def_readonly("solves", &FlowPlan::solves)
      .def_readonly("feasible", &FlowPlan::feasible)
      .def_readonly("solver", &FlowPlan::solver)
      .def_readonly("lp_pivots", &FlowPlan::lp_pivots)
      .def_readonly("lp_status", &FlowPlan::lp_status)
      .def_readonly("jobs", &FlowPlan::jobs);
  m.def("solve_flow", [](const std::map<NodeID, LayerIDs>& holdings,
                         const std::vector<std::tuple<LayerID, NodeID, int64_t>>& demands,
                         const std::map<NodeID, int64_t>& egress, const std::map<NodeID, int64_t>& ingress,
                         const std::map<std::pair<NodeID, NodeID>, int64_t>& links, int64_t align,
                         bool integer_seconds, bool allow_self, const std::map<NodeID, int64_t>& stage,
                         bool stage_once, const std::map<NodeID, int>& disk_group,
                         const std::map<int, int64_t>& disk_group_bps, const std::string& solver,
                         const std::map<NodeID, int>& host, const std::map<NodeID, int64_t>& nic) {
    FlowProblem p;
    p.host = host;
    p.nic_bps = nic;
    p.stage_bps = stage;
    p.stage_once = stage_once;
    p.disk_group = disk_group;
    p.disk_group_bps = disk_group_bps;
    p.solver = solver;
    p.holdings = holdings;
    for (auto& d : demands) p.demands.push_back({std::get<0>(d), std::get<1>(d), std::get<2>(d)});
    p.egress_bps = egress;
    p.ingress_bps = ingress;
    p.link_bps = links;
    p.align = align;
    p.integer_seconds = integer_seconds;
    p.allow_self = allow_self;
    py::gil_scoped_release nogil;
    return solve_flow(p);
  }, py::arg("holdings"), py::arg("demands"), py::arg("egress") = std::map<NodeID, int64_t>{},
     py::arg("ingress") = std::map<NodeID, int64_t>{},
     py::arg("links") = std::map<std::pair<NodeID, NodeID>, int64_t>{}, py::arg("align") = 1,
     py::arg("integer_seconds") = false, py::arg("allow_self") = false,
     py::arg("stage") = std::map<NodeID, int64_t>{}, py::arg("stage_once") = false,
     py::arg("disk_group") = std::map<NodeID, int>{}, py::arg("disk_group_bps") = std::map<int, int64_t>{},
     py::arg("solver") = "auto", py::arg("host") = std::map<NodeID, int>{},
     py::arg("nic") = std::map<NodeID, int64_t>{});

  // Dense two-phase simplex (sched/lp.h); rows as lists of ((col, coef) pairs, rhs).
  m.def("solve_lp", [](int n, const std::vector<double>& c,
                       const std::vector<std::pair<std::vector<std::pair<int, double>>, double>>& eq,
                       const std::vector<std::pair<std::vector<std::pair<int, double>>, double>>& le) {
    LpProblem p;
    p.n = n;
    p.c = c;
    for (auto& r : eq) p.eq.push_back(LpRow{r.first, r.second});
    for (auto& r : le) p.le.push_back(LpRow{r.first, r.second});
    LpResult r = solve_lp(p);
    return py::make_tuple(r.ok, r.status, r.obj, r.x, r.pivots);
  }, py::arg("n"), py::arg("c"), py::arg("eq"), py::arg("le"));

  py::class_<RangeSet>(m, "RangeSet")
      .def(py::init<>())
      .def("add", &RangeSet::add)
      .def("covered", &RangeSet::covered)
      .def("contains", &RangeSet::contains)
      .def("ranges", &RangeSet::ranges);

  // ---- GPU runtime (HIP kernels, device store, RCCL engine): csrc/gpu/
  register_gpu_bindings(m.ptr());
}
