// md5_mb.h -- whole-file MD5s of many files at once on the host (md5_mb.cpp: multi-buffer AVX-512 / AVX2).
#pragma once
#include <stdint.h>

#include "rsync_hip.h"

namespace rsh {

struct Md5File {
    const rsh_piece* pieces;  // the file is the concatenation of its pieces
    int32_t npieces;
};

// MD5 of every file into out[f], on up to `threads` threads.  force_width (tests, A/B): 1 = scalar, 8 = AVX2,
// 16 = AVX-512 (capped at what the CPU has); 0 = the widest the CPU has.
void md5_files(const Md5File* files, int32_t nfiles, uint8_t (*out)[16], int threads, int force_width = 0);
// Lanes of the widest multi-buffer MD5 this CPU runs (16, 8, or 1 for the scalar form).
int md5_simd_width();

}  // namespace rsh
