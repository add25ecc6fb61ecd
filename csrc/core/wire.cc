#include "core/wire.h"

#include <cstdlib>
#include <cstring>
#include <sstream>

namespace dissem {

const char* location_name(Location l) {
  switch (l) {
    case Location::Inmem: return "inmem";
    case Location::Disk: return "disk";
    case Location::Client: return "client";
    case Location::Device: return "device";
  }
  return "?";
}

std::shared_ptr<HostBuffer> HostBuffer::alloc(int64_t size, bool zero) {
  auto b = std::make_shared<HostBuffer>();
  b->size = size;
  size_t n = size_t(size > 0 ? size : 1);
  void* p = zero ? calloc(1, n) : malloc(n);
  if (!p) throw std::bad_alloc();
  b->ptr = static_cast<uint8_t*>(p);
  b->owner = std::shared_ptr<void>(p, free);
  return b;
}

std::shared_ptr<HostBuffer> HostBuffer::wrap(uint8_t* p, int64_t size, std::shared_ptr<void> owner) {
  auto b = std::make_shared<HostBuffer>();
  b->ptr = p;
  b->size = size;
  b->owner = std::move(owner);
  return b;
}

const char* msg_type_name(MsgType t) {
  switch (t) {
    case MsgType::Announce: return "announce";
    case MsgType::Ack: return "ack";
    case MsgType::Layer: return "layer";
    case MsgType::Retransmit: return "retransmit";
    case MsgType::FlowRetransmit: return "flow_retransmit";
    case MsgType::ClientReq: return "client_req";
    case MsgType::Startup: return "startup";
    case MsgType::Simple: return "simple";
    case MsgType::Transport: return "transport";
    case MsgType::Nack: return "nack";
    case MsgType::Bcast: return "bcast";
    case MsgType::XferBatch: return "xfer_batch";
    case MsgType::Suspect: return "suspect";
    case MsgType::Shrink: return "shrink";
    case MsgType::ShrinkDone: return "shrink_done";
    case MsgType::Landed: return "landed";
    case MsgType::SendDone: return "send_done";
    case MsgType::Tick: return "tick";
    case MsgType::Stop: return "stop";
  }
  return "?";
}

std::string node_str(NodeID id) { return std::to_string(id); }

namespace {
std::string to_hex(const std::string& b) {
  static const char* d = "0123456789abcdef";
  std::string out;
  out.reserve(b.size() * 2);
  for (unsigned char c : b) {
    out.push_back(d[c >> 4]);
    out.push_back(d[c & 15]);
  }
  return out;
}
std::string from_hex(const std::string& h) {
  auto v = [](char c) { return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10; };
  std::string out;
  for (size_t i = 0; i + 1 < h.size(); i += 2) out.push_back(char((v(h[i]) << 4) | v(h[i + 1])));
  return out;
}
}  // namespace

NodeID parse_node_id(const std::string& s) {
  char* end = nullptr;
  unsigned long long v = strtoull(s.c_str(), &end, 10);
  if (s.empty() || (end && *end)) throw std::runtime_error("bad node id: " + s);
  return NodeID(v);
}

std::string Message::str() const {
  std::ostringstream o;
  switch (type) {
    case MsgType::Announce: {
      o << src << ": [";
      bool first = true;
      for (auto& kv : layers) {
        o << (first ? "" : " ") << kv.first;
        first = false;
      }
      o << "]";
      break;
    }
    case MsgType::Ack: o << src << ": " << layer; break;
    case MsgType::Retransmit: o << "from " << src << ": layer " << layer << ", to " << dest << ", "; break;
    case MsgType::FlowRetransmit:
      o << "from " << src << ": layer " << layer << ", to " << dest << ", size: " << data_size
        << ", offset: " << offset << ", rate: " << rate;
      break;
    case MsgType::Layer:
      o << "from " << src << ": layer " << layer << ", location: " << int(location) << ", rate: " << rate;
      break;
    case MsgType::ClientReq: o << "from " << src << ": layer " << layer; break;
    case MsgType::Startup: o << "from " << src << ": startup"; break;
    case MsgType::Simple: o << src_addr << ": " << payload_str; break;
    default: o << msg_type_name(type) << " from " << src << " layer " << layer; break;
  }
  return o.str();
}

static Json layer_ids_json(const LayerIDs& ids) {
  Json obj = Json::object();
  for (auto& kv : ids) {
    Json m = Json::object();
    m["Location"] = Json(unsigned(kv.second.location));
    m["LimitRate"] = Json(kv.second.limit_rate);
    m["SourceType"] = Json(unsigned(kv.second.source_type));
    if (kv.second.size) m["DataSize"] = Json(kv.second.size);
    obj[std::to_string(kv.first)] = m;
  }
  return obj;
}

static LayerIDs layer_ids_from(const Json* j) {
  LayerIDs out;
  if (!j || !j->is_object()) return out;
  for (auto& kv : j->as_object()) {
    LayerMeta meta;
    if (kv.second.is_object()) {
      meta.location = Location(kv.second.get_u64("Location", 0));
      meta.limit_rate = kv.second.get_i64("LimitRate", 0);
      meta.source_type = SourceType(kv.second.get_u64("SourceType", 0));
      meta.size = kv.second.get_i64("DataSize", 0);
    }
    out[LayerID(strtoull(kv.first.c_str(), nullptr, 10))] = meta;
  }
  return out;
}

Json encode_layer_header(const Message& m) {
  Json h = Json::object();
  h["SrcID"] = Json(uint64_t(m.src));
  h["LayerID"] = Json(uint64_t(m.layer));
  h["LayerSize"] = Json(m.data_size);
  h["TotalSize"] = Json(m.total_size);
  h["Offert"] = Json(m.offset);  // sic: reference field name (transport.go:52)
  if (m.epoch) h["Epoch"] = Json(uint64_t(m.epoch));
  if (m.chunk_bytes) h["ChunkBytes"] = Json(m.chunk_bytes);
  if (m.seq) h["Seq"] = Json(uint64_t(m.seq));
  if (m.rate) h["Rate"] = Json(m.rate);
  if (!m.crc.empty()) {
    Json arr = Json::array();
    for (uint32_t c : m.crc) arr.push_back(Json(unsigned(c)));
    h["Crc"] = arr;
  }
  return h;
}

Json encode_payload(const Message& m) {
  Json p = Json::object();
  auto src_id = [&] { p["SrcID"] = Json(uint64_t(m.src)); };
  switch (m.type) {
    case MsgType::Announce:
      src_id();
      p["LayerIDs"] = layer_ids_json(m.layers);
      if (!m.manifest.empty()) {
        Json man = Json::object();
        for (auto& kv : m.manifest) {
          Json e = Json::array();
          e.push_back(Json(kv.second.chunk_bytes));
          Json c = Json::array();
          for (uint32_t x : kv.second.crc) c.push_back(Json(unsigned(x)));
          e.push_back(c);
          man[std::to_string(kv.first)] = e;
        }
        p["Manifest"] = man;
      }
      if (!m.link_rates.empty()) {  // measured outbound link rates (B/s), closed-loop planning
        Json lr = Json::object();
        for (auto& kv : m.link_rates) lr[std::to_string(kv.first)] = Json(kv.second);
        p["LinkRates"] = lr;
      }
      if (!m.partial_layers.empty()) {
        Json part = Json::object();
        for (auto& kv : m.partial_layers) {
          Json rs = Json::array();
          for (auto& r : kv.second) {
            Json e = Json::array();
            e.push_back(Json(r.first));
            e.push_back(Json(r.second));
            rs.push_back(e);
          }
          part[std::to_string(kv.first)] = rs;
        }
        p["Partial"] = part;
      }
      break;
    case MsgType::XferBatch: {
      src_id();
      p["Batch"] = Json(uint64_t(m.batch));
      Json arr = Json::array();
      for (auto& j : m.jobs) {
        Json e = Json::array();
        e.push_back(Json(uint64_t(j.seq)));
        e.push_back(Json(uint64_t(j.src)));
        e.push_back(Json(uint64_t(j.dst)));
        e.push_back(Json(uint64_t(j.layer)));
        e.push_back(Json(j.offset));
        e.push_back(Json(j.size));
        e.push_back(Json(j.total));
        e.push_back(Json(j.chunk_bytes));
        Json c = Json::array();
        for (uint32_t x : j.crc) c.push_back(Json(unsigned(x)));
        e.push_back(c);
        if (j.rate) e.push_back(Json(j.rate));
        arr.push_back(e);
      }
      p["Jobs"] = arr;
      break;
    }
    case MsgType::Ack:
      src_id();
      p["LayerID"] = Json(uint64_t(m.layer));
      p["Location"] = Json(unsigned(m.location));  // extension (unexported in reference)
      if (m.partial) {  // extension: a range of the layer landed (mode-2 range jobs)
        p["Partial"] = Json(true);
        p["Offset"] = Json(m.offset);
        p["DataSize"] = Json(m.data_size);
      }
      break;
    case MsgType::Retransmit:
      src_id();
      p["LayerID"] = Json(uint64_t(m.layer));
      p["DestID"] = Json(uint64_t(m.dest));
      break;
    case MsgType::FlowRetransmit:
      src_id();
      p["LayerID"] = Json(uint64_t(m.layer));
      p["DestID"] = Json(uint64_t(m.dest));
      p["DataSize"] = Json(m.data_size);
      p["Offset"] = Json(m.offset);
      p["Rate"] = Json(m.rate);
      break;
    case MsgType::ClientReq:
      src_id();
      p["LayerID"] = Json(uint64_t(m.layer));
      p["SaveDisk"] = Json(m.save_disk);
      break;
    case MsgType::Startup:
      src_id();
      break;
    case MsgType::Simple:
      p["SrcAddr"] = Json(m.src_addr);
      p["PayloadStr"] = Json(m.payload_str);
      break;
    case MsgType::Layer:
      return encode_layer_header(m);
    case MsgType::Nack:
      src_id();
      p["LayerID"] = Json(uint64_t(m.layer));
      p["DestID"] = Json(uint64_t(m.dest));
      p["DataSize"] = Json(m.data_size);
      p["Offset"] = Json(m.offset);
      break;
    case MsgType::Bcast: {
      src_id();
      p["LayerID"] = Json(uint64_t(m.layer));
      p["TotalSize"] = Json(m.total_size);
      p["Seq"] = Json(uint64_t(m.seq));
      p["ChunkBytes"] = Json(m.chunk_bytes);
      Json arr = Json::array();
      for (auto n : m.peers) arr.push_back(Json(uint64_t(n)));
      p["Peers"] = arr;
      if (!m.crc.empty()) {
        Json c = Json::array();
        for (uint32_t x : m.crc) c.push_back(Json(unsigned(x)));
        p["Crc"] = c;
      }
      break;
    }
    case MsgType::Suspect:
    case MsgType::Shrink:
    case MsgType::ShrinkDone: {
      src_id();
      p["Seq"] = Json(uint64_t(m.seq));
      Json arr = Json::array();
      for (auto n : m.peers) arr.push_back(Json(uint64_t(n)));
      p["Peers"] = arr;
      if (!m.payload_str.empty()) p["CommId"] = Json(to_hex(m.payload_str));
      break;
    }
    default:
      throw std::runtime_error(std::string("cannot serialize internal message ") + msg_type_name(m.type));
  }
  if (m.epoch) p["Epoch"] = Json(uint64_t(m.epoch));
  return p;
}

std::string encode_envelope(const Message& m) {
  Json env = Json::object();
  env["type"] = Json(unsigned(m.type));
  env["src"] = Json(m.type == MsgType::Simple ? m.src_addr : node_str(m.src));
  env["payload"] = encode_payload(m);
  return env.dump();
}

MessagePtr decode_envelope(const Json& env) {
  auto m = std::make_shared<Message>();
  if (!env.is_object()) throw std::runtime_error("envelope is not an object");
  m->type = MsgType(env.get_u64("type", 255));
  m->src_str = env.get_str("src");
  const Json* pp = env.find("payload");
  static const Json kEmpty = Json::object();
  const Json& p = (pp && pp->is_object()) ? *pp : kEmpty;
  m->src = p.get_u64("SrcID", 0);
  m->epoch = p.get_u64("Epoch", 0);
  switch (m->type) {
    case MsgType::Announce:
      m->layers = layer_ids_from(p.find("LayerIDs"));
      if (auto* man = p.find("Manifest"); man && man->is_object()) {
        for (auto& kv : man->as_object()) {
          const auto& e = kv.second.as_array();
          CrcManifest cm;
          cm.chunk_bytes = e.at(0).as_i64();
          for (auto& x : e.at(1).as_array()) cm.crc.push_back(uint32_t(x.as_u64()));
          m->manifest[LayerID(strtoull(kv.first.c_str(), nullptr, 10))] = cm;
        }
      }
      if (auto* part = p.find("Partial"); part && part->is_object()) {
        for (auto& kv : part->as_object()) {
          auto& rs = m->partial_layers[LayerID(strtoull(kv.first.c_str(), nullptr, 10))];
          for (auto& e : kv.second.as_array()) rs.push_back({e.as_array().at(0).as_i64(), e.as_array().at(1).as_i64()});
        }
      }
      if (auto* lr = p.find("LinkRates"); lr && lr->is_object())
        for (auto& kv : lr->as_object()) m->link_rates[NodeID(strtoull(kv.first.c_str(), nullptr, 10))] = kv.second.as_i64();
      break;
    case MsgType::XferBatch:
      m->batch = p.get_u64("Batch");
      if (auto* arr = p.find("Jobs"); arr && arr->is_array()) {
        for (auto& e : arr->as_array()) {
          const auto& a = e.as_array();
          XferJob j;
          j.seq = a.at(0).as_u64();
          j.src = a.at(1).as_u64();
          j.dst = a.at(2).as_u64();
          j.layer = a.at(3).as_u64();
          j.offset = a.at(4).as_i64();
          j.size = a.at(5).as_i64();
          j.total = a.at(6).as_i64();
          j.chunk_bytes = a.at(7).as_i64();
          for (auto& x : a.at(8).as_array()) j.crc.push_back(uint32_t(x.as_u64()));
          if (a.size() > 9) j.rate = a.at(9).as_i64();
          m->jobs.push_back(std::move(j));
        }
      }
      break;
    case MsgType::Ack:
      m->layer = p.get_u64("LayerID");
      m->location = Location(p.get_u64("Location", 0));
      m->partial = p.get_bool("Partial", false);
      if (m->partial) {
        m->offset = p.get_i64("Offset", 0);
        m->data_size = p.get_i64("DataSize", 0);
      }
      break;
    case MsgType::Retransmit:
      m->layer = p.get_u64("LayerID");
      m->dest = p.get_u64("DestID");
      break;
    case MsgType::FlowRetransmit:
    case MsgType::Nack:
      m->layer = p.get_u64("LayerID");
      m->dest = p.get_u64("DestID");
      m->data_size = p.get_i64("DataSize");
      m->offset = p.get_i64("Offset");
      m->rate = p.get_i64("Rate");
      break;
    case MsgType::ClientReq:
      m->layer = p.get_u64("LayerID");
      m->save_disk = p.get_bool("SaveDisk");
      break;
    case MsgType::Startup:
      break;
    case MsgType::Simple:
      m->src_addr = p.get_str("SrcAddr");
      m->payload_str = p.get_str("PayloadStr");
      break;
    case MsgType::Layer: {
      m->layer = p.get_u64("LayerID");
      m->data_size = p.get_i64("LayerSize");
      m->total_size = p.get_i64("TotalSize");
      m->offset = p.get_i64("Offert", p.get_i64("Offset", 0));
      m->chunk_bytes = p.get_i64("ChunkBytes", 0);
      m->seq = p.get_u64("Seq", 0);
      m->rate = p.get_i64("Rate", 0);
      if (auto* c = p.find("Crc"); c && c->is_array())
        for (auto& x : c->as_array()) m->crc.push_back(uint32_t(x.as_u64()));
      break;
    }
    case MsgType::Bcast: {
      m->layer = p.get_u64("LayerID");
      m->total_size = p.get_i64("TotalSize");
      m->seq = p.get_u64("Seq");
      m->chunk_bytes = p.get_i64("ChunkBytes");
      if (auto* a = p.find("Peers"); a && a->is_array())
        for (auto& x : a->as_array()) m->peers.push_back(x.as_u64());
      if (auto* c = p.find("Crc"); c && c->is_array())
        for (auto& x : c->as_array()) m->crc.push_back(uint32_t(x.as_u64()));
      break;
    }
    case MsgType::Suspect:
    case MsgType::Shrink:
    case MsgType::ShrinkDone:
      m->seq = p.get_u64("Seq", 0);
      if (auto* a = p.find("Peers"); a && a->is_array())
        for (auto& x : a->as_array()) m->peers.push_back(x.as_u64());
      m->payload_str = from_hex(p.get_str("CommId"));
      break;
    default:
      throw std::runtime_error("unknown MsgType: " + std::to_string(unsigned(m->type)));
  }
  return m;
}

}  // namespace dissem
