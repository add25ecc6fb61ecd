// Core data model (reference: distributor/node.go:128-211, client.go:10).
//
// IDs are 64-bit like Go's `uint` on amd64; ClientID is MaxUint. A layer's
// `Location` gains a fourth tier, Device (HBM), which is the placement target on
// MI355X: the reference's "InmemLayer" is host RAM because it has no GPU.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

namespace dissem {

using NodeID = uint64_t;
using LayerID = uint64_t;
constexpr NodeID kClientID = ~uint64_t(0);  // client.go:10
// XferJob destination meaning "every rank of the data-plane communicator": a
// collective broadcast from the job's src (ncclBroadcast on the GPU).
constexpr NodeID kAllRanks = ~uint64_t(0) - 1;

enum class Location : uint8_t {
  Inmem = 0,   // host RAM (reference InmemLayer)
  Disk = 1,    // file on local storage (reference DiskLayer)
  Client = 2,  // held by an external rate-limited client process (reference ClientLayer)
  Device = 3,  // HBM of this rank's GPU (MI355X extension)
};

enum class SourceType : uint8_t {
  Client = 0,  // node.go:192-198
  Disk = 1,
  Mem = 2,
  Device = 3,  // extension: layer seeded directly in HBM
};

const char* location_name(Location l);

struct LayerMeta {
  Location location = Location::Inmem;
  int64_t limit_rate = 0;  // bytes/s, 0 = unlimited (reference quirk Q1 fixed)
  SourceType source_type = SourceType::Client;
  int64_t size = 0;        // extension: layer bytes, so the leader can plan without holding it (Q8)
};

using LayerIDs = std::map<LayerID, LayerMeta>;   // node.go:141
using Assignment = std::map<NodeID, LayerIDs>;   // node.go:174
using Status = std::map<NodeID, LayerIDs>;       // node.go:176
using NodeIDs = std::set<NodeID>;                // node.go:132

// Host byte buffer with a custom deleter so pinned (hipHostMalloc) memory and
// plain malloc'd memory share one type.
struct HostBuffer {
  uint8_t* ptr = nullptr;
  int64_t size = 0;
  std::shared_ptr<void> owner;  // releases the memory
  static std::shared_ptr<HostBuffer> alloc(int64_t size, bool zero = true);
  static std::shared_ptr<HostBuffer> wrap(uint8_t* p, int64_t size, std::shared_ptr<void> owner);
};

// Where the bytes of a layer live (node.go:200-211), plus device residency.
struct LayerSrc {
  std::shared_ptr<HostBuffer> host;  // host bytes (full layer) or nullptr
  std::string path;                  // disk file or ""
  uint8_t* dev = nullptr;            // HBM bytes (full layer) or nullptr
  int64_t data_size = 0;             // full layer size
  int64_t offset = 0;
  LayerMeta meta;
  // Non-empty: only these [start, end) bytes of the layer are held (a copy
  // resumed at chunk granularity from --persist-dir); not an owner of the rest.
  std::vector<std::pair<int64_t, int64_t>> ranges;
};
using LayersSrc = std::map<LayerID, LayerSrc>;
using PartialLayers = std::map<LayerID, std::vector<std::pair<int64_t, int64_t>>>;

}  // namespace dissem
