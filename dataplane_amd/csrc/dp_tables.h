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

// Validate + lower the descriptors; returns 0 or a negative errno.
int build_image(const dp_tables_desc_t *desc, BuiltImage &out);

}  // namespace dpd
