// host_md5.h -- streaming MD5 on the host (whole-file digest of Sender.java:1241,1326 and the rare
// single resolver windows).  Same compression function as the kernels (md5_core.h).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "md5_core.h"

static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "host MD5 loads message words as little-endian");

namespace rsh {

class HostMd5 {
  public:
    HostMd5() { reset(); }
    void reset() {
        st_ = md5_init();
        nbytes_ = 0;
        nbuf_ = 0;
    }
    void update(const uint8_t* p, size_t n) {
        nbytes_ += n;
        if (nbuf_) {
            size_t take = 64 - nbuf_ < n ? 64 - nbuf_ : n;
            memcpy(buf_ + nbuf_, p, take);
            nbuf_ += take;
            p += take;
            n -= take;
            if (nbuf_ < 64) return;
            block(buf_);
            nbuf_ = 0;
        }
        while (n >= 64) {
            block(p);
            p += 64;
            n -= 64;
        }
        if (n) {
            memcpy(buf_, p, n);
            nbuf_ = n;
        }
    }
    void final(uint8_t out[16]) {
        const uint64_t bits = nbytes_ * 8;
        uint8_t pad[72] = {0x80};
        const size_t padlen = (nbuf_ < 56) ? 56 - nbuf_ : 120 - nbuf_;
        update(pad, padlen);
        uint8_t len[8];
        for (int i = 0; i < 8; i++) len[i] = (uint8_t)(bits >> (8 * i));
        update(len, 8);
        md5_digest_bytes(st_, out);
        reset();
    }

  private:
    void block(const uint8_t* p) {
        uint32_t m[16];
        memcpy(m, p, 64);  // MD5 words are little-endian, as is every host this builds for
        md5_compress(st_, m);
    }
    Md5State st_;
    uint64_t nbytes_;
    uint8_t buf_[64];
    size_t nbuf_;
};

}  // namespace rsh
