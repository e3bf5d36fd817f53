// SPDX-License-Identifier: Apache-2.0
// Host table compiler interface (dp_tables.cpp).
#pragma once
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "../../include/dpgpu.h"
#include "dp_device.h"

namespace dpd {

// A masquerade expose as the tables hold it (dp_masq_expose_t, validated):
// one family, private and public prefixes, the port-forwarding claims on its
// public range.
struct MasqExpose {
  uint32_t src_vni, dst_vni;
  uint64_t idle_ns;
  int fam;
  std::vector<dp_prefix_t> priv, pub;
  std::vector<dp_masq_claim_t> claims;
};
// MasqueradeConfig: the exposes, their canonical bytes and the caller's tag
// (a flow table's allocator is kept across publishes of the same config,
// nat/src/masquerade/allocator_writer.rs:120-154).  The allocator itself is
// flow-table state (dp_masq.h), built from this when a table syncs.
struct MasqConfig {
  std::vector<MasqExpose> exposes;
  std::string canon;
  uint64_t tag = 0;
  bool randomize = false;  // MasqueradeConfig::set_randomize, and the permutations' seed
  uint64_t seed = 0;
  bool same(const MasqConfig &o) const {
    if (randomize != o.randomize || seed != o.seed) return false;
    return tag || o.tag ? tag == o.tag && o.tag != 0 : canon == o.canon;
  }
};

struct BuiltImage {
  std::vector<uint8_t> bytes;  // host copy of the device image
  Image im;                    // offsets into `bytes`
  uint64_t pt_nodes = 0;
  std::shared_ptr<const MasqConfig> masq;  // never null after a successful build
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
