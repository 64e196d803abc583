// wav.cpp — host-side RIFF/WAVE reader of libhfa: the front end of tools/load_wav.py:4-8 (torchaudio.load with its
// default normalize=True).  PCM 8/16/24/32-bit integer and IEEE float 32/64, plain or WAVE_FORMAT_EXTENSIBLE,
// scaled as torchaudio does: uint8 (x - 128) / 128, int16 / 2^15, 24-bit / 2^23, int32 / 2^31, float64 rounded to
// float32.  One channel (or all, planar) is decoded straight into the caller's buffer — e.g. a row of the pinned
// batch buffer infer.py uploads — so the CLI keeps only the batch in flight in memory, not the whole folder.
// Plain C stdio, no shared state: the calls are re-entrant (infer.py reads a batch's files on a thread pool; ctypes
// drops the GIL for the call) and never touch the GPU.
#include "hfa_common.h"

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <exception>
#include <vector>

namespace {

struct WavFmt {
    int tag = 0, channels = 0, rate = 0, bits = 0, block = 0;
    long long data_off = -1, data_bytes = 0;
};

inline uint32_t rd32(const unsigned char* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
inline uint16_t rd16(const unsigned char* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

struct File {
    FILE* f = nullptr;
    explicit File(const char* path) : f(fopen(path, "rb")) {}
    ~File() {
        if (f) fclose(f);
    }
};

// Walks the chunk list (headers only; the data chunk is skipped) -> 0, or HFA_EINVAL with the error set.
int parse(File& fh, const char* path, WavFmt& w) {
    if (!fh.f) {
        hfa::set_error("hfa_wav: cannot open %s", path);
        return HFA_EINVAL;
    }
    unsigned char head[12];
    if (fread(head, 1, 12, fh.f) != 12 || memcmp(head, "RIFF", 4) || memcmp(head + 8, "WAVE", 4)) {
        hfa::set_error("hfa_wav: %s: not a RIFF/WAVE file", path);
        return HFA_EINVAL;
    }
    long long pos = 12;
    bool have_fmt = false;
    unsigned char hdr[8];
    while (fread(hdr, 1, 8, fh.f) == 8) {
        const uint32_t size = rd32(hdr + 4);
        const long long body = pos + 8, next = body + size + (size & 1);
        if (!memcmp(hdr, "fmt ", 4)) {
            unsigned char b[40] = {0};
            const size_t want = size < sizeof(b) ? size : sizeof(b);
            if (size < 16 || fread(b, 1, want, fh.f) != want) {
                hfa::set_error("hfa_wav: %s: short fmt chunk", path);
                return HFA_EINVAL;
            }
            w.tag = rd16(b);
            w.channels = rd16(b + 2);
            w.rate = (int)rd32(b + 4);
            w.block = rd16(b + 12);
            w.bits = rd16(b + 14);
            if (w.tag == 0xFFFE && size >= 26) w.tag = rd16(b + 24);   // WAVE_FORMAT_EXTENSIBLE: the sub-format
            have_fmt = true;
        } else if (!memcmp(hdr, "data", 4)) {
            w.data_off = body;
            w.data_bytes = size;
        }
        if (have_fmt && w.data_off >= 0) break;
        if (fseeko(fh.f, next, SEEK_SET) != 0) break;
        pos = next;
    }
    if (!have_fmt || w.data_off < 0) {
        hfa::set_error("hfa_wav: %s: missing fmt or data chunk", path);
        return HFA_EINVAL;
    }
    // a data chunk that claims more than the file holds (streaming writers: 0xFFFFFFFF) ends at the end of file
    if (fseeko(fh.f, 0, SEEK_END) == 0) {
        const long long avail = (long long)ftello(fh.f) - w.data_off;
        if (avail < w.data_bytes) w.data_bytes = avail > 0 ? avail : 0;
    }
    const bool pcm = w.tag == 1 && (w.bits == 8 || w.bits == 16 || w.bits == 24 || w.bits == 32);
    const bool flt = w.tag == 3 && (w.bits == 32 || w.bits == 64);
    if (!pcm && !flt) {
        hfa::set_error("hfa_wav: %s: unsupported format tag %d / %d bits", path, w.tag, w.bits);
        return HFA_EINVAL;
    }
    if (w.channels < 1 || w.rate < 1) {
        hfa::set_error("hfa_wav: %s: %d channels at %d Hz", path, w.channels, w.rate);
        return HFA_EINVAL;
    }
    return 0;
}

static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "RIFF samples are little-endian; so is the host");

// one sample, scaled as torchaudio.load(normalize=True)
template <int TAG, int BITS>
inline float sample(const unsigned char* p) {
    if constexpr (TAG == 3 && BITS == 32) {
        float v;
        memcpy(&v, p, 4);
        return v;
    } else if constexpr (TAG == 3) {
        double v;
        memcpy(&v, p, 8);
        return (float)v;
    } else if constexpr (BITS == 8) {
        return ((float)p[0] - 128.0f) / 128.0f;
    } else if constexpr (BITS == 16) {
        int16_t v;                                   // little-endian host (static_assert above): a plain load
        memcpy(&v, p, 2);
        return (float)v * (1.0f / 32768.0f);
    } else if constexpr (BITS == 24) {
        int32_t v = (int32_t)(p[0] | (p[1] << 8) | (p[2] << 16));
        if (v >= (1 << 23)) v -= (1 << 24);
        return (float)v * (1.0f / 8388608.0f);
    } else {
        int32_t v;
        memcpy(&v, p, 4);
        return (float)v * (1.0f / 2147483648.0f);    // round to f32, then exact scaling
    }
}

// m interleaved frames of ch channels (frames f0.. of n) -> dst: one channel, or all of them planar (channel -1)
template <int TAG, int BITS>
void decode(const unsigned char* b, long long m, int ch, int channel, long long f0, long long n, float* dst) {
    constexpr int bps = BITS / 8;
    if (ch == 1) {                                   // mono: contiguous, vectorised
        float* __restrict__ d = dst + f0;
        for (long long i = 0; i < m; ++i) d[i] = sample<TAG, BITS>(b + i * bps);
        return;
    }
    const int c0 = channel >= 0 ? channel : 0, c1 = channel >= 0 ? channel + 1 : ch;
    for (int c = c0; c < c1; ++c) {                  // one channel at a time: a strided gather per channel
        float* __restrict__ d = dst + (channel >= 0 ? 0 : (long long)c * n) + f0;
        const unsigned char* s = b + (long long)c * bps;
        for (long long i = 0; i < m; ++i) d[i] = sample<TAG, BITS>(s + i * ch * bps);
    }
}

}  // namespace

extern "C" {

int hfa_wav_info(const char* path, int64_t* frames, int32_t* channels, int32_t* sample_rate) {
    if (!path || !frames || !channels || !sample_rate) {
        hfa::set_error("hfa_wav_info: null argument");
        return HFA_EINVAL;
    }
    File fh(path);
    WavFmt w;
    if (int rc = parse(fh, path, w)) return rc;
    const int bps = w.bits / 8;
    *frames = w.data_bytes / ((long long)bps * w.channels);
    *channels = w.channels;
    *sample_rate = w.rate;
    return 0;
}

static int wav_read(const char* path, int32_t channel, float* dst, int64_t capacity, int64_t* frames,
                    int32_t* sample_rate) {
    if (!path || !dst || !frames || capacity < 0) {
        hfa::set_error("hfa_wav_read: null argument or negative capacity");
        return HFA_EINVAL;
    }
    File fh(path);
    WavFmt w;
    if (int rc = parse(fh, path, w)) return rc;
    if (channel < -1 || channel >= w.channels) {
        hfa::set_error("hfa_wav_read: %s: channel %d of %d", path, channel, w.channels);
        return HFA_EINVAL;
    }
    const int bps = w.bits / 8, ch = w.channels;
    const long long n = w.data_bytes / ((long long)bps * ch);
    const long long need = channel < 0 ? n * ch : n;
    if (need > capacity) {
        hfa::set_error("hfa_wav_read: %s: %lld samples do not fit a buffer of %lld", path, need, (long long)capacity);
        return HFA_EINVAL;
    }
    // decode in blocks of whole frames through a small staging buffer (no copy of the whole data chunk), at most
    // 64 Ki frames and 4 MiB whatever the header's channel count and sample width claim
    constexpr long long kBudget = 4ll << 20;
    const long long frame_bytes = (long long)bps * ch;
    long long kBlock = kBudget / frame_bytes < (1 << 16) ? kBudget / frame_bytes : (1 << 16);
    if (kBlock > n) kBlock = n;
    if (kBlock < 1) kBlock = 1;
    std::vector<unsigned char> buf((size_t)(kBlock * frame_bytes));
    if (fseeko(fh.f, w.data_off, SEEK_SET) != 0) {
        hfa::set_error("hfa_wav_read: %s: seek failed", path);
        return HFA_EINVAL;
    }
    for (long long f0 = 0; f0 < n; f0 += kBlock) {
        const long long m = n - f0 < kBlock ? n - f0 : kBlock;
        if (fread(buf.data(), 1, (size_t)(m * bps * ch), fh.f) != (size_t)(m * bps * ch)) {
            hfa::set_error("hfa_wav_read: %s: truncated data chunk", path);
            return HFA_EINVAL;
        }
        const unsigned char* b = buf.data();
        if (w.tag == 3 && w.bits == 32) decode<3, 32>(b, m, ch, channel, f0, n, dst);
        else if (w.tag == 3) decode<3, 64>(b, m, ch, channel, f0, n, dst);
        else if (w.bits == 8) decode<1, 8>(b, m, ch, channel, f0, n, dst);
        else if (w.bits == 16) decode<1, 16>(b, m, ch, channel, f0, n, dst);
        else if (w.bits == 24) decode<1, 24>(b, m, ch, channel, f0, n, dst);
        else decode<1, 32>(b, m, ch, channel, f0, n, dst);
    }
    *frames = n;
    if (sample_rate) *sample_rate = w.rate;
    return 0;
}

int hfa_wav_read(const char* path, int32_t channel, float* dst, int64_t capacity, int64_t* frames,
                 int32_t* sample_rate) {
    try {                                            // nothing may unwind through the C ABI (ctypes callers)
        return wav_read(path, channel, dst, capacity, frames, sample_rate);
    } catch (const std::exception& e) {
        hfa::set_error("hfa_wav_read: %s: %s", path ? path : "(null)", e.what());
        return HFA_EINVAL;
    }
}

}  // extern "C"
