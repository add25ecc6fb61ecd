#include "core/wire.h"

#include <charconv>
#include <string_view>

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
      if (!m.link_rates_in.empty()) {  // inbound links timed at the receiving end
        Json lr = Json::object();
        for (auto& kv : m.link_rates_in) lr[std::to_string(kv.first)] = Json(kv.second);
        p["LinkRatesIn"] = lr;
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
      if (m.order) p["Order"] = Json(uint64_t(m.order));
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
        std::string hx(j.crc.size() * 8, '0');
        for (size_t i = 0; i < j.crc.size(); ++i) {
          static const char* dg = "0123456789abcdef";
          for (int k = 0; k < 8; ++k) hx[i * 8 + size_t(k)] = dg[(j.crc[i] >> (4 * (7 - k))) & 15];
        }
        e.push_back(Json(hx));
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

namespace {
// Transfer batches are the largest control messages (every job of a session,
// each with its chunks' CRCs) and sit between "timer start" and the first
// byte on a link: written straight to text, the same bytes the Json DOM
// dump gives (sorted keys: envelope payload/src/type, payload Batch/Epoch/Jobs/SrcID).
// Writes into a buffer sized for the worst case up front (no per-append checks).
struct Out {
  char* p;
  template <class T>
  void num(T v) {
    p = std::to_chars(p, p + 24, v).ptr;
  }
  void lit(const char* t) {
    const size_t n = strlen(t);
    memcpy(p, t, n);
    p += n;
  }
  void ch(char c) { *p++ = c; }
  // CRCs as one string of 8 hex digits each (a job's chunk CRCs are most of a
  // batch: fixed-width hex is ~10x cheaper to write and read than decimals)
  void hex(const std::vector<uint32_t>& v) {
    static const char* d = "0123456789abcdef";
    for (uint32_t x : v)
      for (int k = 7; k >= 0; --k) *p++ = d[(x >> (4 * k)) & 15];
  }
};

std::string encode_xfer_batch(const Message& m) {
  size_t crcs = 0;
  for (auto& j : m.jobs) crcs += j.crc.size();
  std::string s;
  s.resize(128 + m.jobs.size() * (10 * 21 + 8) + crcs * 8);
  Out o{s.data()};
  o.lit("{\"payload\":{\"Batch\":");
  o.num(uint64_t(m.batch));
  if (m.epoch) {
    o.lit(",\"Epoch\":");
    o.num(uint64_t(m.epoch));
  }
  o.lit(",\"Jobs\":[");
  for (size_t i = 0; i < m.jobs.size(); ++i) {
    const XferJob& j = m.jobs[i];
    if (i) o.ch(',');
    o.ch('[');
    o.num(uint64_t(j.seq));
    o.ch(',');
    o.num(uint64_t(j.src));
    o.ch(',');
    o.num(uint64_t(j.dst));
    o.ch(',');
    o.num(uint64_t(j.layer));
    o.ch(',');
    o.num(j.offset);
    o.ch(',');
    o.num(j.size);
    o.ch(',');
    o.num(j.total);
    o.ch(',');
    o.num(j.chunk_bytes);
    o.ch(',');
    o.ch('"');
    o.hex(j.crc);
    o.ch('"');
    if (j.rate) {
      o.ch(',');
      o.num(j.rate);
    }
    o.ch(']');
  }
  o.lit("]");
  if (m.order) {
    o.lit(",\"Order\":");
    o.num(uint64_t(m.order));
  }
  o.lit(",\"SrcID\":");
  o.num(uint64_t(m.src));
  o.lit("},\"src\":\"");
  o.num(uint64_t(m.src));
  o.lit("\",\"type\":");
  o.num(uint64_t(unsigned(m.type)));
  o.ch('}');
  s.resize(size_t(o.p - s.data()));
  return s;
}

bool parse_crc_hex(std::string_view h, std::vector<uint32_t>* out) {
  if (h.size() % 8) return false;
  out->reserve(h.size() / 8);
  for (size_t i = 0; i < h.size(); i += 8) {
    uint32_t v = 0;
    for (size_t k = 0; k < 8; ++k) {
      const char c = h[i + k];
      uint32_t d;
      if (c >= '0' && c <= '9') d = uint32_t(c - '0');
      else if (c >= 'a' && c <= 'f') d = uint32_t(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') d = uint32_t(c - 'A' + 10);
      else return false;
      v = (v << 4) | d;
    }
    out->push_back(v);
  }
  return true;
}

// A cursor over envelope text for the transfer-batch fast path. Any shape it
// does not expect makes it give up (ok = false): the caller then decodes the
// same bytes through the Json DOM, so it only ever saves time.
struct Cur {
  const char* p;
  const char* e;
  bool ok = true;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool eat(char c) {
    ws();
    if (p < e && *p == c) {
      ++p;
      return true;
    }
    return false;
  }
  void need(char c) {
    if (!eat(c)) ok = false;
  }
  bool key(std::string_view* k) {  // "name" then ':'
    ws();
    if (p >= e || *p != '"') return ok = false;
    const char* b = ++p;
    while (p < e && *p != '"') {
      if (*p == '\\') return ok = false;
      ++p;
    }
    if (p >= e) return ok = false;
    *k = std::string_view(b, size_t(p - b));
    ++p;
    need(':');
    return ok;
  }
  template <class T>
  T num() {
    ws();
    T v{};
    auto r = std::from_chars(p, e, v);
    if (r.ec != std::errc()) {
      ok = false;
      return T{};
    }
    p = r.ptr;
    return v;
  }
  // skip one value of any kind (strings, numbers, nested containers)
  void skip() {
    ws();
    size_t n = Json::scan_prefix(p, size_t(e - p));
    if (n == 0) ok = false;
    p += n;
  }
};

bool decode_xfer_payload(Cur& c, Message& m) {
  if (!c.eat('{')) return false;
  if (c.eat('}')) return true;
  do {
    std::string_view k;
    if (!c.key(&k)) return false;
    if (k == "Batch") {
      m.batch = c.num<uint64_t>();
    } else if (k == "Epoch") {
      m.epoch = c.num<uint64_t>();
    } else if (k == "Order") {
      m.order = c.num<uint8_t>();
    } else if (k == "SrcID") {
      m.src = c.num<uint64_t>();
    } else if (k == "Jobs") {
      if (!c.eat('[')) return false;
      m.jobs.reserve(256);
      if (!c.eat(']')) {
        do {
          XferJob j;
          if (!c.eat('[')) return false;
          j.seq = c.num<uint64_t>();
          c.need(',');
          j.src = c.num<uint64_t>();
          c.need(',');
          j.dst = c.num<uint64_t>();
          c.need(',');
          j.layer = c.num<uint64_t>();
          c.need(',');
          j.offset = c.num<int64_t>();
          c.need(',');
          j.size = c.num<int64_t>();
          c.need(',');
          j.total = c.num<int64_t>();
          c.need(',');
          j.chunk_bytes = c.num<int64_t>();
          c.need(',');
          if (c.eat('"')) {
            const char* b = c.p;
            while (c.p < c.e && *c.p != '"') ++c.p;
            if (c.p >= c.e || !parse_crc_hex(std::string_view(b, size_t(c.p - b)), &j.crc)) return false;
            ++c.p;
          } else {
            if (!c.eat('[')) return false;
            if (!c.eat(']')) {
              do j.crc.push_back(c.num<uint32_t>());
              while (c.ok && c.eat(','));
              c.need(']');
            }
          }
          if (c.eat(',')) j.rate = c.num<int64_t>();
          c.need(']');
          if (!c.ok) return false;
          m.jobs.push_back(std::move(j));
        } while (c.eat(','));
        c.need(']');
      }
    } else {
      return false;  // a field this path does not know: the DOM decoder handles it
    }
  } while (c.ok && c.eat(','));
  c.need('}');
  return c.ok;
}
}  // namespace

MessagePtr decode_envelope_text(const char* buf, size_t len) {
  {
    Cur c{buf, buf + len};
    auto m = std::make_shared<Message>();
    bool batch = false, typed = false;
    if (c.eat('{') && !c.eat('}')) {
      do {
        std::string_view k;
        if (!c.key(&k)) break;
        if (k == "payload") {
          batch = decode_xfer_payload(c, *m);
          if (!batch) break;
        } else if (k == "src") {
          c.ws();
          c.skip();  // "src" is informative: SrcID in the payload is the sender
        } else if (k == "type") {
          typed = c.num<unsigned>() == unsigned(MsgType::XferBatch);
          if (!typed) break;
        } else {
          c.ok = false;
        }
      } while (c.ok && c.eat(','));
      if (batch && typed && c.ok && c.eat('}')) {
        m->type = MsgType::XferBatch;
        m->src_str = node_str(m->src);
        return m;
      }
    }
  }
  return decode_envelope(Json::parse(std::string(buf, len)));
}

std::string encode_envelope(const Message& m) {
  if (m.type == MsgType::XferBatch) return encode_xfer_batch(m);
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
      if (auto* lr = p.find("LinkRatesIn"); lr && lr->is_object())
        for (auto& kv : lr->as_object())
          m->link_rates_in[NodeID(strtoull(kv.first.c_str(), nullptr, 10))] = kv.second.as_i64();
      break;
    case MsgType::XferBatch:
      m->batch = p.get_u64("Batch");
      m->order = uint8_t(p.get_u64("Order", 0));
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
          if (a.at(8).is_string()) {
            if (!parse_crc_hex(a.at(8).as_str(), &j.crc)) throw std::runtime_error("bad CRC hex in xfer job");
          } else {
            for (auto& x : a.at(8).as_array()) j.crc.push_back(uint32_t(x.as_u64()));
          }
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
