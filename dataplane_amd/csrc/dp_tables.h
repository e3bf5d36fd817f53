// SPDX-License-Identifier: Apache-2.0
// Host table compiler interface (dp_tables.cpp).
#pragma once
#include <stdint.h>

#include <vector>

#include "../../include/dpgpu.h"
#include "dp_device.h"

namespace dpd {

struct BuiltImage {
  std::vector<uint8_t> bytes;  // host copy of the device image
  Image im;                    // offsets into `bytes`
  uint64_t pt_nodes = 0;
};

// The port-forwarding entries of a device's current generation (the lineage
// PortFwTable::update carries from one publish to the next).
struct PfEntry {
  dp_portfw_rule_t r;
  uint32_t id;
};
struct PfLineage {
  std::vector<PfEntry> live;
  uint32_t next_id = 1;
};

// Validate + lower the descriptors; returns 0 or a negative errno.  `pf`:
// the device's port-forwarding lineage, updated with the new rule set (only
// when the build succeeds).
int build_image(const dp_tables_desc_t *desc, BuiltImage &out, PfLineage *pf = nullptr);

}  // namespace dpd
