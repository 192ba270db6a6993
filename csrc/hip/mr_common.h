// mr_common.h — shared device/host definitions for the MI355X MapReduce kernels.
//
// Key model (replaces the reference's interned Lua string/tuple keys,
// /root/reference/mapreduce/tuple.lua:121-140 and the string keys emitted by
// examples/WordCount/mapfn.lua:4-7):
//
//   Every key is a 128-bit value (hi, lo):
//     * len <= 15  ("packed", exact):  hi = bytes[0..7] big-endian,
//                                     lo = bytes[8..14] big-endian << 8 | len
//       -> (hi, lo) compared as unsigned 128-bit == byte-lexicographic order
//          (the order Lua's string `<` gives, utils.lua:126).
//     * len >= 16  ("long", hashed):   hi = bytes[0..7] big-endian (exact prefix),
//                                     lo = hash56(bytes) << 8 | 0xFF
//       -> (prefix, 56-bit hash) selects the slot; identity is EXACT: a table
//          insert that matches a long key on (hi, lo) compares the key bytes
//          through the rep words (hashtab.h), so colliding keys stay apart.
//   lo is never 0, so lo == 0 marks an unwritten table slot.
//
//   A "rep" word locates the key bytes of a long key inside a byte source:
//       rep = (offset << 24) | min(len, 2^24-1)
#pragma once
#include <stdint.h>

#ifndef MR_HD
#if defined(__HIPCC__)
#define MR_HD __host__ __device__ __forceinline__
#else
#define MR_HD inline
#endif
#endif

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint8_t u8;
typedef uint16_t u16;

namespace mr {

constexpr u64 LONG_MARK = 0xFFull;
constexpr int PACK_MAX = 15;          // longest exactly-packed key
constexpr u64 REP_LEN_BITS = 24;
constexpr u64 REP_LEN_MASK = (1ull << REP_LEN_BITS) - 1;

// Lua 5.2 "%s" in the C locale: \t \n \v \f \r and space
// (examples/WordCount/mapfn.lua:5 uses "[^%s]+").
MR_HD bool is_ws(u32 c) { return c == 32u || (c - 9u) < 5u; }

MR_HD u64 fmix64(u64 x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// Slot tag of a key: never 0 (0 marks an empty slot).
MR_HD u64 key_tag(u64 hi, u64 lo) { return fmix64(hi ^ fmix64(lo + 0x9E3779B97F4A7C15ull)) | 1ull; }

// Claim word of a key in the HBM table (hashtab.h).  A packed key of at most
// 7 bytes has lo == len (1..7) and zero low byte in hi, so hi | lo IS the key:
// claiming its slot publishes the key in one atomic and a tag match is a key
// match (no wait for the claimer's payload stores).  These are the frequent
// words of natural text, whose slots every workgroup hits at once on a cold
// table.  Other keys get a 56-bit hash with low byte 0x80 (never an exact tag).
MR_HD bool gtab_tag_exact(u64 tag) { return (tag & 0xF8ull) == 0; }
MR_HD u64 gtab_tag(u64 hi, u64 lo) {
  // (generic callers may insert arbitrary (hi, lo): the exact form is used only
  // where it is injective — 1 <= lo <= 7 and a zero low byte in hi)
  return (lo - 1 < 7 && (hi & 0xFFull) == 0) ? (hi | lo)
                                             : ((fmix64(hi ^ fmix64(lo + 0x9E3779B97F4A7C15ull)) & ~0xFFull) | 0x80ull);
}
MR_HD u64 gtab_home(u64 tag, u64 mask) { return fmix64(tag ^ 0x2545F4914F6CDD1Dull) & mask; }

// Hash of a long key, word-at-a-time over little-endian 8-byte words (the last
// one zero padded).  Identical on host and device.
MR_HD u64 long_hash_step(u64 h, u64 w) { return fmix64(h ^ w) * 0x9E3779B97F4A7C15ull; }
MR_HD u64 long_hash_init(u64 len) { return 0x243F6A8885A308D3ull ^ (len * 0x13198A2E03707344ull); }
// `mask` keeps the low bits of the 56-bit hash: all of them in production; a
// debug knob (mr_set_long_mask_*, ops.set_long_hash_bits) truncates it so that
// distinct long keys collide and the byte verification of the tables is tested.
MR_HD u64 long_lo(u64 h, u64 mask) { return ((fmix64(h) & mask) << 8) | LONG_MARK; }

#if defined(__HIPCC__)
// Per translation unit (no -fgpu-rdc): the long-key hash mask read by its
// kernels and the host setter of that copy.
#define MR_LONG_MASK_SYMBOL(tu)                                                        \
  static __constant__ u64 mr_long_mask = ~0ull;                                         \
  extern "C" int mr_set_long_mask_##tu(u64 m) {                                         \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(mr_long_mask), &m, sizeof(m));              \
  }
#endif

MR_HD bool key_is_long(u64 lo) { return (lo & 0xFFull) == LONG_MARK; }
MR_HD u32 packed_len(u64 lo) { return (u32)(lo & 0xFFull); }

// Byte i (0-based) of a packed key.
MR_HD u32 packed_byte(u64 hi, u64 lo, u32 i) {
  return i < 8 ? (u32)((hi >> (56 - 8 * i)) & 0xFF) : (u32)((lo >> (56 - 8 * (i - 8))) & 0xFF);
}

// Exact uint32 FNV-1 (multiply, then xor), the hash of the reference
// partitionfn (examples/WordCount/partitionfn.lua:8-16).  The reference computes
// it in Lua doubles, which drops low bits once h*prime exceeds 2^53; this is the
// exact 32-bit form (documented difference).
constexpr u32 FNV_PRIME = 16777619u;
constexpr u32 FNV_OFFSET = 2166136261u;
MR_HD u32 fnv1_step(u32 h, u32 b) { return (h * FNV_PRIME) ^ b; }

// Two keys' bytes (rep words into one byte source) are equal.  The bytes are
// compared 16 at a time with every load of a batch issued before the first
// compare (a byte loop with an early exit waits out one memory round trip
// per byte on the device: n-gram keys of 20-40 bytes that hit in the table).
MR_HD bool rep_bytes_equal(const u8* src, u64 a, u64 b) {
  const u64 n = a & REP_LEN_MASK;
  if (n != (b & REP_LEN_MASK)) return false;
  const u64 oa = a >> REP_LEN_BITS, ob = b >> REP_LEN_BITS;
  if (oa == ob) return true;
  for (u64 i = 0; i < n; i += 16) {
    u32 diff = 0;
#pragma unroll
    for (u64 j = 0; j < 16; ++j)
      if (i + j < n) diff |= (u32)(src[oa + i + j] ^ src[ob + i + j]);
    if (diff) return false;
  }
  return true;
}

// Row index read from a sort permutation, clamped into [0, n): a radix pass
// whose look-back gave up (flagged, the result is discarded and re-sorted)
// may leave stale permutation entries, which must never become an
// out-of-bounds read in the gathers that follow.
MR_HD u64 clamp_row(u64 j, u64 n) { return j < n ? j : 0; }

MR_HD u64 make_rep(u64 off, u64 len) { return (off << REP_LEN_BITS) | (len < REP_LEN_MASK ? len : REP_LEN_MASK); }
MR_HD u64 rep_off(u64 rep) { return rep >> REP_LEN_BITS; }
MR_HD u64 rep_len(u64 rep) { return rep & REP_LEN_MASK; }

// Copy n bytes of a key from global memory, 16 loads in flight per batch (a
// byte loop waits out one memory round trip per byte: n-gram keys of 16-40
// bytes).
MR_HD void copy_key_bytes(u8* dst, const u8* p, u64 n) {
  for (u64 k0 = 0; k0 < n; k0 += 16) {
    u8 b[16];
#pragma unroll
    for (u64 j = 0; j < 16; ++j) b[j] = k0 + j < n ? p[k0 + j] : (u8)0;
#pragma unroll
    for (u64 j = 0; j < 16; ++j)
      if (k0 + j < n) dst[k0 + j] = b[j];
  }
}

// Little-endian word of bytes p[0 .. min(n, 8)) (zero past the end), its
// loads issued together (long-key hash words).
MR_HD u64 load_word_le(const u8* p, u64 n) {
  u64 w = 0;
#pragma unroll
  for (u64 j = 0; j < 8; ++j) w |= (j < n ? (u64)p[j] : 0ull) << (8 * j);
  return w;
}

// FNV-1 of a table key's bytes (packed in (hi, lo), or at rep in src for a
// long key) and its length.
MR_HD u32 key_fnv(u64 h, u64 l, u64 r, const u8* src, u32* len_out) {
  u32 f = FNV_OFFSET;
  u32 len;
  if (!key_is_long(l)) {
    len = packed_len(l);
    for (u32 k = 0; k < len; ++k) f = fnv1_step(f, packed_byte(h, l, k));
  } else {
    len = (u32)rep_len(r);
    const u8* p = src + rep_off(r);
    for (u32 k0 = 0; k0 < len; k0 += 16) {  // 16 loads in flight per batch
      u32 b[16];
#pragma unroll
      for (u32 j = 0; j < 16; ++j) b[j] = k0 + j < len ? (u32)p[k0 + j] : 0u;
#pragma unroll
      for (u32 j = 0; j < 16; ++j)
        if (k0 + j < len) f = fnv1_step(f, b[j]);
    }
  }
  *len_out = len;
  return f;
}

// Reduction operators for hash aggregation / reduce-by-key.
// OP_NONE: the table only maps keys to slots (a vocabulary: the inverted
// index's word ids) — inserts fold nothing, so a hit costs one load, no atomic.
enum ReduceOp : int { OP_SUM = 0, OP_MIN = 1, OP_MAX = 2, OP_COUNT = 3, OP_NONE = 4 };

}  // namespace mr
