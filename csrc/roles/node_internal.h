// Helpers shared by the Node's translation units (node.cc: lifecycle,
// receiver, sender, failure handling; mode01.cc, mode2.cc, mode3.cc: the
// leader's schedulers; multihost.cc: the multi-host planners).
#pragma once

#include "core/types.h"

namespace dissem {

// Does `ids` hold layer `l` in tier location `loc`?
inline bool at(const LayerIDs& ids, LayerID l, Location loc) {
  auto it = ids.find(l);
  return it != ids.end() && it->second.location == loc;
}

}  // namespace dissem
