// Per-node layer store: where each layer's bytes live and which byte ranges of
// an incoming layer have landed (reference: LayersSrc map guarded by the role's
// RWMutex, node.go:166,200-211; partial assembly node.go:1520-1567).
//
// Differences by design: fragments are assembled at their
// offset, and completion is decided by a coverage set, so a layer completes
// exactly once no matter how many senders stripe it or how often a range is
// re-sent.
#pragma once

#include <map>
#include <mutex>
#include <vector>

#include "core/types.h"

namespace dissem {

// Disjoint [start, end) byte ranges.
class RangeSet {
 public:
  // Adds [a, b); returns the number of newly covered bytes.
  int64_t add(int64_t a, int64_t b);
  int64_t covered() const { return covered_; }
  bool contains(int64_t a, int64_t b) const;
  void clear() {
    r_.clear();
    covered_ = 0;
  }
  std::vector<std::pair<int64_t, int64_t>> ranges() const { return {r_.begin(), r_.end()}; }

 private:
  std::map<int64_t, int64_t> r_;
  int64_t covered_ = 0;
};

struct Slot {
  LayerSrc src;            // src.meta.location = best tier where the layer is complete
  bool has_target = false; // complete in the node's target tier
  RangeSet landed;         // coverage of an in-progress target-tier copy
  int64_t total = 0;
  bool acked = false;
};

class LayerStore {
 public:
  LayerStore(const LayersSrc& init, Location target);

  Location target() const { return target_; }
  // Inventory for Announce: {layer: {Location, LimitRate, SourceType, DataSize}}.
  LayerIDs inventory();
  // Layers held only in part (resumed chunk ranges), for Announce's Partial.
  PartialLayers partial();
  bool get(LayerID id, LayerSrc* out);
  bool has_target(LayerID id);
  void put(LayerID id, const LayerSrc& src);
  std::vector<LayerID> ids();

  // Host landing area for a layer (allocated on first use, full layer size).
  uint8_t* host_landing(LayerID id, int64_t total);
  // Device slot pointer for a layer, if the GPU store provisioned one.
  uint8_t* device_slot(LayerID id);
  void set_device_slot(LayerID id, uint8_t* p, int64_t total);

  // Records that [off, off+size) is now resident in the target tier.
  // Returns true exactly once: when the layer becomes complete.
  bool mark_landed(LayerID id, int64_t off, int64_t size, int64_t total);
  int64_t landed_bytes(LayerID id);

  // Drops target-tier copies that were not part of the initial inventory
  // (used to re-run a dissemination session on the same store).
  void reset_to(const LayersSrc& init);

  std::mutex mu;  // guards slots_

 private:
  Location target_;
  std::map<LayerID, Slot> slots_;
};

// Disk-tier layer files and this OS's page cache (reference: conf/exe.sh:17
// drops every cache before a run). file_cache_drop writes back and evicts the
// file's cached pages (fdatasync + POSIX_FADV_DONTNEED); both return the
// fraction of the file's pages still resident (mincore), so a benchmark can
// show its reads did not come from memory. -1: the file could not be mapped.
double file_cache_drop(const std::string& path);
double file_cache_resident(const std::string& path);

}  // namespace dissem
