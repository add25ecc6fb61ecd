#include "store/store.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace dissem {

int64_t RangeSet::add(int64_t a, int64_t b) {
  if (b <= a) return 0;
  int64_t before = covered_;
  // Merge with every overlapping/adjacent range.
  auto it = r_.upper_bound(a);
  if (it != r_.begin()) {
    auto prev = std::prev(it);
    if (prev->second >= a) it = prev;
  }
  int64_t na = a, nb = b;
  while (it != r_.end() && it->first <= nb) {
    na = std::min(na, it->first);
    nb = std::max(nb, it->second);
    covered_ -= it->second - it->first;
    it = r_.erase(it);
  }
  r_[na] = nb;
  covered_ += nb - na;
  return covered_ - before;
}

bool RangeSet::contains(int64_t a, int64_t b) const {
  if (b <= a) return true;
  auto it = r_.upper_bound(a);
  if (it == r_.begin()) return false;
  --it;
  return it->first <= a && it->second >= b;
}

LayerStore::LayerStore(const LayersSrc& init, Location target) : target_(target) { reset_to(init); }

void LayerStore::reset_to(const LayersSrc& init) {
  std::lock_guard<std::mutex> lk(mu);
  // Keep provisioned device slots (they are reused across sessions).
  std::map<LayerID, std::pair<uint8_t*, int64_t>> dev;
  for (auto& kv : slots_)
    if (kv.second.src.dev) dev[kv.first] = {kv.second.src.dev, kv.second.total};
  slots_.clear();
  for (auto& kv : init) {
    Slot s;
    s.src = kv.second;
    s.total = kv.second.data_size;
    s.src.meta.size = kv.second.data_size;
    s.has_target = kv.second.meta.location == target_;
    if (s.has_target) s.landed.add(0, s.total);
    slots_[kv.first] = s;
  }
  for (auto& kv : dev) {
    Slot& s = slots_[kv.first];
    s.src.dev = kv.second.first;
    if (!s.total) s.total = kv.second.second;
  }
}

LayerIDs LayerStore::inventory() {
  std::lock_guard<std::mutex> lk(mu);
  LayerIDs out;
  for (auto& kv : slots_) {
    const Slot& s = kv.second;
    // A provisioned-but-empty device slot is not an inventory entry.
    if (!s.has_target && !s.src.host && s.src.path.empty() && s.src.meta.location != Location::Client)
      continue;
    if (!s.has_target && !s.src.ranges.empty()) continue;  // partial copy: announced separately
    LayerMeta m = s.src.meta;
    m.size = s.total;
    if (s.has_target) m.location = target_;
    out[kv.first] = m;
  }
  return out;
}

PartialLayers LayerStore::partial() {
  std::lock_guard<std::mutex> lk(mu);
  PartialLayers out;
  for (auto& kv : slots_)
    if (!kv.second.has_target && !kv.second.src.ranges.empty()) out[kv.first] = kv.second.src.ranges;
  return out;
}

bool LayerStore::get(LayerID id, LayerSrc* out) {
  std::lock_guard<std::mutex> lk(mu);
  auto it = slots_.find(id);
  if (it == slots_.end()) return false;
  *out = it->second.src;
  out->data_size = it->second.total;
  if (it->second.has_target) out->meta.location = target_;
  return true;
}

bool LayerStore::has_target(LayerID id) {
  std::lock_guard<std::mutex> lk(mu);
  auto it = slots_.find(id);
  return it != slots_.end() && it->second.has_target;
}

void LayerStore::put(LayerID id, const LayerSrc& src) {
  std::lock_guard<std::mutex> lk(mu);
  Slot& s = slots_[id];
  uint8_t* dev = s.src.dev;
  s.src = src;
  if (!s.src.dev) s.src.dev = dev;
  s.total = src.data_size;
  s.has_target = src.meta.location == target_;
  s.landed.clear();
  if (s.has_target) s.landed.add(0, s.total);
}

std::vector<LayerID> LayerStore::ids() {
  std::lock_guard<std::mutex> lk(mu);
  std::vector<LayerID> out;
  for (auto& kv : slots_) out.push_back(kv.first);
  return out;
}

uint8_t* LayerStore::host_landing(LayerID id, int64_t total) {
  std::lock_guard<std::mutex> lk(mu);
  Slot& s = slots_[id];
  if (!s.total) s.total = total;
  if (s.total != total) throw std::runtime_error("layer " + std::to_string(id) + " size mismatch");
  if (!s.src.host || s.src.host->size < total) {
    // The fresh landing copy replaces any lower-tier reference for this layer.
    s.src.host = HostBuffer::alloc(total, false);
  }
  return s.src.host->ptr;
}

uint8_t* LayerStore::device_slot(LayerID id) {
  std::lock_guard<std::mutex> lk(mu);
  auto it = slots_.find(id);
  return it == slots_.end() ? nullptr : it->second.src.dev;
}

void LayerStore::set_device_slot(LayerID id, uint8_t* p, int64_t total) {
  std::lock_guard<std::mutex> lk(mu);
  Slot& s = slots_[id];
  s.src.dev = p;
  if (!s.total) s.total = total;
}

bool LayerStore::mark_landed(LayerID id, int64_t off, int64_t size, int64_t total) {
  std::lock_guard<std::mutex> lk(mu);
  Slot& s = slots_[id];
  if (!s.total) s.total = total;
  if (s.has_target) return false;
  s.landed.add(off, off + size);
  if (s.landed.covered() >= s.total) {
    s.has_target = true;
    s.src.data_size = s.total;
    s.src.meta.location = target_;
    s.src.meta.size = s.total;
    return true;
  }
  return false;
}

int64_t LayerStore::landed_bytes(LayerID id) {
  std::lock_guard<std::mutex> lk(mu);
  auto it = slots_.find(id);
  return it == slots_.end() ? 0 : it->second.landed.covered();
}

double file_cache_resident(const std::string& path) {
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -1;
  struct stat st {};
  double frac = -1;
  if (fstat(fd, &st) == 0 && st.st_size > 0) {
    void* p = mmap(nullptr, size_t(st.st_size), PROT_READ, MAP_SHARED, fd, 0);
    if (p != MAP_FAILED) {
      const long page = sysconf(_SC_PAGESIZE);
      const size_t pages = (size_t(st.st_size) + size_t(page) - 1) / size_t(page);
      std::vector<unsigned char> v(pages);
      if (mincore(p, size_t(st.st_size), v.data()) == 0) {
        size_t in = 0;
        for (unsigned char b : v) in += b & 1;
        frac = double(in) / double(pages);
      }
      munmap(p, size_t(st.st_size));
    }
  } else if (st.st_size == 0) {
    frac = 0;
  }
  ::close(fd);
  return frac;
}

double file_cache_drop(const std::string& path) {
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -1;
  (void)fdatasync(fd);  // dirty pages cannot be dropped
  (void)posix_fadvise(fd, 0, 0, POSIX_FADV_DONTNEED);
  ::close(fd);
  return file_cache_resident(path);
}

}  // namespace dissem
