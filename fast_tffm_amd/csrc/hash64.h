// MurmurHash64A with the seed TensorFlow's Hash64() uses (0xDECAFCAFFE).
//
// Parity target: reference cc/fm_parser_op.cc:82-84 hashes the feature-id token
// with tensorflow::Hash64(p, len) and takes it modulo vocab_size; the reference
// test (test/fm_parser_op_test.py:30-46) compares that against
// tf.string_to_hash_bucket, i.e. the same function. Bit-exact here, usable from
// host code (parser) and from device code (synthetic data / GPU tokenizer).
#pragma once
#include <cstdint>
#include <cstddef>

#if defined(__HIPCC__)
#define FM_HD __host__ __device__ inline
#else
#define FM_HD inline
#endif

namespace fm {

constexpr uint64_t kHash64Seed = 0xDECAFCAFFEull;

FM_HD uint64_t hash64(const char* data, size_t n, uint64_t seed = kHash64Seed) {
  const uint64_t m = 0xc6a4a7935bd1e995ull;
  const int r = 47;
  uint64_t h = seed ^ (static_cast<uint64_t>(n) * m);
  while (n >= 8) {
    uint64_t k = 0;
    for (int b = 0; b < 8; ++b)  // little-endian decode, alignment-free
      k |= static_cast<uint64_t>(static_cast<unsigned char>(data[b])) << (8 * b);
    data += 8;
    n -= 8;
    k *= m;
    k ^= k >> r;
    k *= m;
    h ^= k;
    h *= m;
  }
  switch (n) {
    case 7: h ^= static_cast<uint64_t>(static_cast<unsigned char>(data[6])) << 48; [[fallthrough]];
    case 6: h ^= static_cast<uint64_t>(static_cast<unsigned char>(data[5])) << 40; [[fallthrough]];
    case 5: h ^= static_cast<uint64_t>(static_cast<unsigned char>(data[4])) << 32; [[fallthrough]];
    case 4: h ^= static_cast<uint64_t>(static_cast<unsigned char>(data[3])) << 24; [[fallthrough]];
    case 3: h ^= static_cast<uint64_t>(static_cast<unsigned char>(data[2])) << 16; [[fallthrough]];
    case 2: h ^= static_cast<uint64_t>(static_cast<unsigned char>(data[1])) << 8; [[fallthrough]];
    case 1:
      h ^= static_cast<uint64_t>(static_cast<unsigned char>(data[0]));
      h *= m;
  }
  h ^= h >> r;
  h *= m;
  h ^= h >> r;
  return h;
}

// 64-bit integer finaliser (splitmix64) used by the synthetic Criteo-shaped
// generator to hash (field, value) pairs into the global slot space.
FM_HD uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

}  // namespace fm
