// Wire protocol: message kinds and the JSON envelope (reference:
// distributor/message.go:16-301, transport.go:47-54).
//
// Every control message is {"type":<u8>,"src":"<id>","payload":{...}} with the
// reference's payload field names, so a capture of our control plane reads like
// the reference's. Extensions are additive fields (Epoch, Location on Ack,
// ChunkBytes/Crc on layer headers) that the reference decoder would ignore.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "core/json.h"
#include "core/types.h"

namespace dissem {

enum class MsgType : uint8_t {
  Announce = 0,
  Ack = 1,
  Layer = 2,
  Retransmit = 3,
  FlowRetransmit = 4,
  ClientReq = 5,
  Startup = 6,
  Simple = 7,
  Transport = 8,
  // ---- extensions ----
  Nack = 9,        // receiver -> sender: chunk CRC mismatch, resend range
  Bcast = 10,      // leader -> participants: collective broadcast descriptor (GPU mode 0)
  XferBatch = 11,  // leader -> ranks: sequence-numbered transfer jobs (GPU planned data plane)
  // Elastic recovery of the planned (RCCL) data plane:
  Suspect = 12,     // rank -> leader: a P2P group with these peers is stuck or failed
  Shrink = 13,      // leader -> survivors: drop these dead nodes from the communicator (Seq = generation)
  ShrinkDone = 14,  // rank -> leader: communicator shrunk, in-flight state reset (Seq = generation)
  // ---- node-internal events (never serialized) ----
  Landed = 32,     // a byte range of a layer is now resident in the target tier
  SendDone = 33,   // a sender finished pushing a range
  Tick = 34,       // periodic timer (watchdogs)
  Stop = 35,       // shut down the event loop
};

const char* msg_type_name(MsgType t);

// One transfer of a byte range of a layer from `src` to `dst` (src == dst: a
// local promotion into HBM). Jobs carry a leader-assigned global sequence
// number; every rank executes its jobs in sequence order, which makes the
// RCCL point-to-point schedule deadlock-free (csrc/engine/planned_engine.cc).
struct XferJob {
  uint64_t seq = 0;
  NodeID src = 0, dst = 0;
  LayerID layer = 0;
  int64_t offset = 0, size = 0, total = 0;
  int64_t chunk_bytes = 0;     // CRC chunk grid of the layer
  std::vector<uint32_t> crc;   // expected CRC32C of the grid chunks the range covers
  int64_t rate = 0;            // pacing of the sends (B/s, 0 = unlimited; mode 3: size/T)
};

// Per-layer integrity manifest announced by holders: CRC32C per chunk.
struct CrcManifest {
  int64_t chunk_bytes = 0;
  std::vector<uint32_t> crc;
};

struct Message {
  MsgType type = MsgType::Simple;
  NodeID src = 0;        // SrcID (payload) - numeric sender id
  std::string src_str;   // envelope "src" as received
  uint64_t epoch = 0;    // session epoch; 0 = legacy (accept)

  // Announce
  LayerIDs layers;
  // Ack / Retransmit / FlowRetransmit / ClientReq / Layer header
  LayerID layer = 0;
  NodeID dest = 0;
  int64_t data_size = 0;   // range bytes (LayerSize in the layer header)
  int64_t offset = 0;
  int64_t rate = 0;
  int64_t total_size = 0;  // full layer size
  Location location = Location::Inmem;
  bool partial = false;    // Ack extension: [offset, offset+data_size) landed (mode-2 range jobs)
  bool save_disk = false;
  // Layer header extensions (GPU data plane)
  int64_t chunk_bytes = 0;
  std::vector<uint32_t> crc;    // expected CRC32C per chunk of the range
  uint64_t seq = 0;             // per (src,dest) stream sequence number
  std::vector<NodeID> peers;    // Bcast participants; Suspect / Shrink node lists
  // XferBatch / Announce extensions
  uint64_t batch = 0;
  // XferBatch: how lanes order its pieces - 0 chunk-major (chunk index, then
  // sequence number: every job of a batch advances chunk by chunk together,
  // as paced mode-3 jobs must), 1 job-major (sequence number, then chunk:
  // mode-2 pull jobs, so a sender's links stay on the layer its copy queue stages)
  uint8_t order = 0;
  std::vector<XferJob> jobs;
  std::map<LayerID, CrcManifest> manifest;
  PartialLayers partial_layers;  // Announce extension: layers held only in these byte ranges
  std::map<NodeID, int64_t> link_rates;  // Announce extension: sender's measured rate to each peer (B/s)
  std::map<NodeID, int64_t> link_rates_in;  // ... and each peer's link INTO the sender, timed at this end (B/s)
  // Simple
  std::string src_addr, payload_str;

  // Host payload for Layer messages: `data` holds the range bytes unless
  // `in_place` (the bytes already sit in the receiver's store slot).
  std::shared_ptr<HostBuffer> data;
  int64_t data_off = 0;  // offset of the range inside `data`
  bool in_place = false;
  double dur_ms = 0;     // internal: transfer duration for logs/throughput

  std::string str() const;  // human readable (message.go String())
};
using MessagePtr = std::shared_ptr<Message>;

Json encode_payload(const Message& m);
// Envelope bytes (no trailing newline, like the reference's conn.Write).
std::string encode_envelope(const Message& m);
// Layer header payload = tempLayerInfo{SrcID, LayerID, LayerSize, TotalSize, Offert} + extensions.
Json encode_layer_header(const Message& m);
// Decode an envelope. Layer envelopes decode into a header-only Layer message.
MessagePtr decode_envelope(const Json& env);
// Decode one envelope's text (exactly one JSON value): transfer batches take a
// direct path, anything else goes through the Json DOM.
MessagePtr decode_envelope_text(const char* buf, size_t len);

std::string node_str(NodeID id);
NodeID parse_node_id(const std::string& s);

}  // namespace dissem
