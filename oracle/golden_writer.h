// golden_writer.h -- TEST INFRASTRUCTURE. Writes the "HVXG" golden container
// read by tests/golden_io.py:
//   magic "HVXG" | u32 narrays | per array: char name[32] | char dtype[8] |
//   u32 ndim | u32 shape[4] | raw little-endian data
#pragma once
#include <cstdio>
#include <cstring>
#include <cstdint>
#include <string>
#include <vector>

struct GoldenArray {
  std::string name, dtype;
  std::vector<uint32_t> shape;
  std::vector<uint8_t> bytes;
};

class GoldenWriter {
 public:
  template <typename T>
  void add(const std::string &name, const char *dtype, const std::vector<uint32_t> &shape,
           const std::vector<T> &data) {
    GoldenArray a;
    a.name = name; a.dtype = dtype; a.shape = shape;
    size_t n = 1;
    for (auto s : shape) n *= s;
    if (n != data.size()) { fprintf(stderr, "golden %s: size mismatch %zu vs %zu\n", name.c_str(), n, data.size()); abort(); }
    a.bytes.resize(n * sizeof(T));
    if (n) memcpy(a.bytes.data(), data.data(), n * sizeof(T));
    arrays.push_back(a);
  }
  void write(const std::string &path) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) { perror(path.c_str()); abort(); }
    fwrite("HVXG", 1, 4, f);
    uint32_t n = arrays.size();
    fwrite(&n, 4, 1, f);
    for (auto &a : arrays) {
      char name[32] = {0}, dt[8] = {0};
      strncpy(name, a.name.c_str(), 31);
      strncpy(dt, a.dtype.c_str(), 7);
      fwrite(name, 1, 32, f); fwrite(dt, 1, 8, f);
      uint32_t nd = a.shape.size(), sh[4] = {1, 1, 1, 1};
      for (uint32_t i = 0; i < nd; i++) sh[i] = a.shape[i];
      fwrite(&nd, 4, 1, f); fwrite(sh, 4, 4, f);
      fwrite(a.bytes.data(), 1, a.bytes.size(), f);
    }
    fclose(f);
    fprintf(stderr, "wrote %s (%zu arrays)\n", path.c_str(), arrays.size());
  }
  std::vector<GoldenArray> arrays;
};

// splitmix64 -- the repo's synthetic-input PRNG
struct SplitMix64 {
  uint64_t s;
  explicit SplitMix64(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  uint32_t u8() { return (uint32_t)(next() >> 56); }
  int range(int lo, int hi) { return lo + (int)(next() % (uint64_t)(hi - lo + 1)); }
};
