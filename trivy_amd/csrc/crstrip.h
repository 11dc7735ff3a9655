// GPU-side CR strip of a packed device batch.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace tsg {

// Device scratch for a strip of `total` bytes (the stripped total is stored
// as a uint64 at the start of it).
size_t cr_strip_scratch_bytes(uint64_t total);

// Enqueue on `s`: dst = src with every '\r' removed, new_off[i] = the
// position of file i's first byte in dst (new_off[nfiles] = stripped total).
// src, dst: 16-byte aligned device buffers of >= total bytes; offsets:
// nfiles + 1 device uint64, nondecreasing, offsets[0] = 0, offsets[nfiles] =
// total.  Wrong offsets give wrong new_off but no access outside the buffers.
bool cr_strip_launch(const uint8_t* src, const uint64_t* offsets, uint32_t nfiles, uint64_t total, uint8_t* dst,
                     uint64_t* new_off, void* scratch, hipStream_t s, std::string* err);

}  // namespace tsg
