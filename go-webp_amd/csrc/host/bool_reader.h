// VP8 boolean entropy decoder (RFC 6386 §7), host side.
//
// Restates the reference's VP8BitReader (pkg/vp8/bits_reader_vp8.go:17-212, the
// libwebp 1.6.0 bit_reader with BITS = 56 on 64-bit hosts): `range` is kept as
// range-1 in [126, 254], `value` is a 64-bit window holding `bits`+8 unread bits,
// bytes are pulled 7 at a time while >= 8 remain and one at a time at the tail
// (VP8LoadNewBytes / VP8LoadFinalBytes, :69-104).  `eof` is set the first time a
// bit is needed past the end of the buffer, exactly as the reference does, since
// the caller's error behaviour (NOT_ENOUGH_DATA) depends on it.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>

namespace wg {

struct BoolReader {
  uint64_t value = 0;
  uint32_t range = 254;  // range - 1
  int bits = -8;         // number of valid bits left
  const uint8_t* buf = nullptr;
  const uint8_t* buf_end = nullptr;
  const uint8_t* buf_max = nullptr;  // last position where an 8-byte load is safe
  int eof = 0;

  void init(const uint8_t* start, size_t size) {  // VP8InitBitReader (:37-46)
    range = 255 - 1;
    value = 0;
    bits = -8;
    eof = 0;
    buf = start;
    buf_end = start + size;
    buf_max = size >= 8 ? start + size - 8 + 1 : start;
    load_new_bytes();
  }

  void load_final_bytes() {  // VP8LoadFinalBytes (:56-69, body per the `// C:` lines)
    if (buf < buf_end) {
      bits += 8;
      value = static_cast<uint64_t>(*buf++) | (value << 8);
    } else if (!eof) {
      value <<= 8;
      bits += 8;
      eof = 1;
    } else {
      bits = 0;  // avoid undefined shifts
    }
  }

  inline void load_new_bytes() {  // VP8LoadNewBytes (:88-113), BITS = 56
    if (buf < buf_max) {
      uint64_t in;
      std::memcpy(&in, buf, 8);
      buf += 7;
      in = __builtin_bswap64(in) >> 8;
      value = in | (value << 56);
      bits += 56;
    } else {
      load_final_bytes();
    }
  }

  inline int get_bit(int prob) {  // VP8GetBit (:116-141)
    uint32_t r = range;
    if (bits < 0) load_new_bytes();
    const int pos = bits;
    const uint32_t split = (r * static_cast<uint32_t>(prob)) >> 8;
    const uint32_t v = static_cast<uint32_t>(value >> pos);
    const int bit = v > split;
    if (bit) {
      r -= split;
      value -= static_cast<uint64_t>(split + 1) << pos;
    } else {
      r = split + 1;
    }
    const int shift = 7 ^ (31 - __builtin_clz(r));  // 7 ^ BitsLog2Floor(range)
    r <<= shift;
    bits -= shift;
    range = r - 1;
    return bit;
  }

  inline int get_signed(int v) {  // VP8GetSigned (:144-160), prob = 0x80
    if (bits < 0) load_new_bytes();
    const int pos = bits;
    const uint32_t split = range >> 1;
    const uint32_t val = static_cast<uint32_t>(value >> pos);
    const int32_t mask = static_cast<int32_t>(split - val) >> 31;  // -1 or 0
    bits -= 1;
    range += static_cast<uint32_t>(mask);
    range |= 1;
    value -= static_cast<uint64_t>((split + 1) & static_cast<uint32_t>(mask)) << pos;
    return (v ^ mask) - mask;
  }

  inline uint32_t get_value(int nbits) {  // VP8GetValue (:72-79)
    uint32_t v = 0;
    while (nbits-- > 0) v |= static_cast<uint32_t>(get_bit(0x80)) << nbits;
    return v;
  }

  inline int get_signed_value(int nbits) {  // VP8GetSignedValue (:82-87)
    const int v = static_cast<int>(get_value(nbits));
    return get_bit(0x80) ? -v : v;
  }
};

}  // namespace wg
