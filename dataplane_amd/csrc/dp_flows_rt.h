// SPDX-License-Identifier: Apache-2.0
//
// Host-side state of a device flow table (include/dpgpu.h "Flow table"),
// shared by the flow-table API (dp_flows.hip) and the burst runtime
// (dp_runtime.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <mutex>

#include "dp_flow.h"
#include "dp_tables.h"

// A device buffer grown on demand and kept (hipFree synchronises the device,
// so it never runs on a call that bursts may overlap).
struct FlowScratch {
  void *p = nullptr;
  size_t cap = 0;
  void *get(size_t bytes) {
    if (bytes <= cap) return p;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    cap = bytes;
    return p;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct dp_flow_table {
  int device = 0;
  dpf::FlowSlot *slots = nullptr;  // HBM
  uint64_t nslots = 0;
  uint32_t mask = 0;
  uint64_t capacity = 0;           // FlowTable::set_capacity
  uint64_t len = 0;                // FULL slots (FlowTable::len)
  uint32_t max_probe = 0;          // largest displacement of any flow ever stored: a lookup
                                   // probes at most max_probe + 1 slots, however many
                                   // tombstones removals have left
  uint32_t *d_meta = nullptr;      // device word: the inserts' atomicMax of their displacement
  hipStream_t stream = nullptr;    // management kernels
  // One order for everything that touches the table: management calls and the
  // flows bursts of every attached context.  A management call holds `mu` for
  // its whole (synchronous) run and first waits for `last_burst`; a flows
  // launch takes `mu`, waits for `last_burst` too (bursts of contexts sharing
  // the table never overlap: their burst-local invalidation marks live in the
  // shared slots) and records `last_burst` after its kernels.
  std::mutex mu;
  hipEvent_t last_burst = nullptr;
  bool burst_armed = false;
  FlowScratch scr[4];              // management-call buffers
  // the masquerade allocator (dp_masq.h): its device buffer (nullptr: none),
  // its generation (the one the flows' allocations name), the config it was
  // built from, the image build the table last synced with, the next
  // generation, the departures' release list
  uint8_t *mq = nullptr;
  uint32_t mq_gen = 0;
  uint32_t mq_next_gen = 1;
  std::shared_ptr<const dpd::MasqConfig> mq_cfg;
  uint64_t mq_serial = 0;
  FlowScratch mq_rel;
  // the release kernels' per-record chain heads and kill list (dp_flows.hip
  // rel_run; all heads kNone between calls), per-entry links; the allocator's
  // address records
  FlowScratch mq_heads, mq_next;
  uint32_t *mq_heads_at = nullptr;
  uint32_t mq_heads_n = 0;
  uint32_t mq_recs = 0;
  // a burst under an image that configures stateful NAT ran on the table (its
  // flows may carry NAT state from then on): bursts keep the full flows variant
  bool snat_seen = false;
};

// update_nat_allocator (nat/src/masquerade/allocator_writer.rs:120-154) for
// one flow table and the published image's masquerade config: the same config
// upgrades the masquerading flows' generation, none drops the allocator and
// invalidates them, a new one replaces the allocator and carries over the
// flows it still serves (check_masquerading_flow, flows.rs:94-174).  Once per
// image build (`serial`); the caller holds ft->mu.  dp_flows.hip.
int dpf_masq_sync(dp_flow_table *ft, const std::shared_ptr<const dpd::MasqConfig> &cfg, int64_t genid,
                  uint64_t serial);
// A destroyed flow table leaves the publish registry (dp_runtime.cpp).
extern "C" void dpr_forget_flow_table(dp_flow_table *ft);

// Error reporting of the library (dp_last_error), defined in dp_runtime.cpp.
int dpr_fail(int rc, const char *what, hipError_t e = hipSuccess);
