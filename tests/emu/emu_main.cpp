// TEST INFRASTRUCTURE (see dp_emu_shim.h).
#include <cstring>
#include <vector>

#include "../../dataplane_amd/csrc/dp_tables.h"

extern "C" void dpemu_run(const uint8_t *img_base, const void *image_struct, uint8_t *buf,
                          uint64_t buf_bytes, const dp_pkt_in_t *in, dp_pkt_out_t *out, uint32_t n);

extern "C" int dpemu_process(const dp_tables_desc_t *d, uint8_t *buf, uint64_t buf_bytes,
                             const dp_pkt_in_t *in, dp_pkt_out_t *out, uint32_t n) {
  dpd::BuiltImage bi;
  int rc = dpd::build_image(d, bi);
  if (rc) return rc;
  uint64_t padded = ((buf_bytes + 15) & ~15ull) + 16;
  std::vector<uint8_t> store(padded + 16);
  uint8_t *al = reinterpret_cast<uint8_t *>(((uintptr_t)store.data() + 15) & ~(uintptr_t)15);
  memcpy(al, buf, buf_bytes);
  // the image is position independent (offsets); align its host copy too
  std::vector<uint8_t> img(bi.bytes.size() + 16);
  uint8_t *ib = reinterpret_cast<uint8_t *>(((uintptr_t)img.data() + 15) & ~(uintptr_t)15);
  memcpy(ib, bi.bytes.data(), bi.bytes.size());
  dpemu_run(ib, &bi.im, al, padded, in, out, n);
  memcpy(buf, al, buf_bytes);
  return 0;
}

extern "C" uint64_t dpemu_image_bytes(const dp_tables_desc_t *d) {
  dpd::BuiltImage bi;
  if (dpd::build_image(d, bi)) return 0;
  return bi.bytes.size();
}
