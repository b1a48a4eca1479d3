// ABI utilities: version, thread-local last-error string.
#include "common.h"
#include <cstdio>

namespace acfe {
static thread_local char g_err[256] = "";
void set_error(hipError_t e, const char* where) {
  std::snprintf(g_err, sizeof(g_err), "%s: %s (%d)", where, hipGetErrorString(e), (int)e);
}
}  // namespace acfe

ACFE_API int acfe_version(void) { return 100; }
ACFE_API const char* acfe_last_error(void) { return acfe::g_err; }

// ---------------------------------------------------------------- host: CRC32C
// Castagnoli CRC (reflected polynomial 0x82F63B78), slicing-by-8, for the
// TFRecord framing (length and data CRCs, masked by the caller).
namespace {
struct Crc32cTables {
  uint32_t t[8][256];
  Crc32cTables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
};
const Crc32cTables& crc_tables() {
  static const Crc32cTables tb;
  return tb;
}
}  // namespace

ACFE_API uint32_t acfe_crc32c(const void* data, size_t n, uint32_t crc) {
  const Crc32cTables& tb = crc_tables();
  const unsigned char* p = static_cast<const unsigned char*>(data);
  crc = ~crc;
  while (n >= 8) {
    uint32_t lo, hi;
    __builtin_memcpy(&lo, p, 4);
    __builtin_memcpy(&hi, p + 4, 4);
    lo ^= crc;
    crc = tb.t[7][lo & 0xFF] ^ tb.t[6][(lo >> 8) & 0xFF] ^ tb.t[5][(lo >> 16) & 0xFF] ^ tb.t[4][lo >> 24] ^
          tb.t[3][hi & 0xFF] ^ tb.t[2][(hi >> 8) & 0xFF] ^ tb.t[1][(hi >> 16) & 0xFF] ^ tb.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) crc = (crc >> 8) ^ tb.t[0][(crc ^ *p++) & 0xFF];
  return ~crc;
}
