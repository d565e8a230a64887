// Host-side helpers of libtde.so (no device code).
//
// tde_crc32c: CRC-32C (Castagnoli, reflected polynomial 0x82F63B78), slicing-by-8, for the TF tensor
// bundle checkpoint format (tf_depth_estimation_amd/checkpoint.py): BundleEntryProto.crc32c of every
// tensor payload and the masked CRC of every index-table block.  Replaces TF's
// tensorflow/core/lib/hash/crc32c used by BundleWriter/BundleReader behind tf.train.Saver
// (batch_prediction.py:49-55, split_training.py:147-202).
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../include/tde.h"

namespace {

struct Crc32cTables {
  uint32_t t[8][256];
  Crc32cTables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
};

const Crc32cTables& tables() {
  static const Crc32cTables tab;
  return tab;
}

}  // namespace

extern "C" uint32_t tde_crc32c(const void* data, size_t n, uint32_t crc) {
  const Crc32cTables& T = tables();
  const unsigned char* p = static_cast<const unsigned char*>(data);
  uint32_t c = crc ^ 0xFFFFFFFFu;
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = T.t[7][lo & 0xFF] ^ T.t[6][(lo >> 8) & 0xFF] ^ T.t[5][(lo >> 16) & 0xFF] ^ T.t[4][lo >> 24] ^
        T.t[3][hi & 0xFF] ^ T.t[2][(hi >> 8) & 0xFF] ^ T.t[1][(hi >> 16) & 0xFF] ^ T.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = T.t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}
