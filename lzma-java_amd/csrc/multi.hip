// multi.hip -- the multi-device batch entry points (SURVEY.md 8(b)'s
// `device_mask`): one host process drives several GPUs of a node without a
// launcher. The streams of a batch are dealt round-robin over the devices
// whose bit is set in the mask (the j-th selected device takes streams
// j, j + D, j + 2D, ... -- SURVEY 8(e)'s {i : i mod G = r}); every device runs
// the single-device path (lzma_enc_batch / lzma_dec_batch) on its own context
// from its own host thread. There is no inter-device exchange: the host
// assembles the outputs in stream order.
#include <algorithm>
#include <cstring>
#include <string>
#include <new>
#include <stdexcept>
#include <thread>
#include <vector>

#include "../../include/lzma_mi355x.h"

struct lzma_mctx {
    uint32_t magic = 0x584D5A4Cu;   // "LZMX" (runtime.h kMctxMagic): first member, checked by every entry point
    std::vector<int> devices;
    std::vector<lzma_ctx*> ctxs;
    std::string err;
};

namespace {

constexpr uint32_t kMagic = 0x584D5A4Cu;
bool valid(const lzma_mctx* m) { return m && m->magic == kMagic; }

int fail(lzma_mctx* m, int code, const std::string& msg) {
    m->err = msg;
    return code;
}

// A worker's exception (std::bad_alloc from a host staging vector, ...) becomes a
// status code in its slot instead of reaching std::terminate in the caller's process.
template <typename F>
void guarded(F&& f, int& rc, std::string& why) {
    try {
        f();
    } catch (const std::bad_alloc&) {
        rc = LZMA_E_NOMEM;
        why = "host staging allocation failed";
    } catch (const std::exception& e) {
        rc = LZMA_E_INTERNAL;
        why = e.what();
    } catch (...) {
        rc = LZMA_E_INTERNAL;
        why = "unknown exception";
    }
}

struct Deal {
    std::vector<std::vector<int>> idx;   // per device: global stream indices
    Deal(int nstreams, int ndev) : idx(ndev) {
        for (int i = 0; i < nstreams; i++) idx[i % ndev].push_back(i);
    }
};

}  // namespace

extern "C" {

int lzma_mctx_create(uint32_t device_mask, lzma_mctx** out) {
    if (!out || device_mask == 0) return LZMA_E_PARAM;
    *out = nullptr;
    lzma_mctx* m = new (std::nothrow) lzma_mctx();
    if (!m) return LZMA_E_NOMEM;
    for (int d = 0; d < 32; d++) {
        if (!(device_mask >> d & 1u)) continue;
        lzma_ctx* c = nullptr;
        int rc = lzma_ctx_create(d, &c);
        if (rc != LZMA_OK) {
            lzma_mctx_destroy(m);
            return rc;
        }
        m->devices.push_back(d);
        m->ctxs.push_back(c);
    }
    *out = m;
    return LZMA_OK;
}

void lzma_mctx_destroy(lzma_mctx* m) {
    if (!valid(m)) return;
    for (lzma_ctx* c : m->ctxs) lzma_ctx_destroy(c);
    m->magic = 0;
    delete m;
}

const char* lzma_mctx_last_error(const lzma_mctx* m) {
    return valid(m) ? m->err.c_str() : "null or invalid multi-device context";
}

int lzma_mctx_devices(const lzma_mctx* m) { return valid(m) ? (int)m->devices.size() : 0; }

int lzma_mctx_set_batch_bytes(lzma_mctx* m, uint64_t bytes) {
    if (!valid(m)) return LZMA_E_PARAM;
    for (lzma_ctx* c : m->ctxs) {
        const int rc = lzma_ctx_set_batch_bytes(c, bytes);
        if (rc != LZMA_OK) return fail(m, rc, "batch bytes must be >= 4096");
    }
    return LZMA_OK;
}

int lzma_mctx_set_timing(lzma_mctx* m, int on) {
    if (!valid(m)) return LZMA_E_PARAM;
    for (lzma_ctx* c : m->ctxs) lzma_ctx_set_timing(c, on);
    return LZMA_OK;
}

int lzma_enc_batch_multi(lzma_mctx* m, const lzma_params* p, const uint8_t* in, const uint64_t* offs, int nstreams,
                         uint8_t* out, uint64_t out_cap, uint64_t* out_offs) {
    if (!valid(m) || !p || !offs || !out_offs || nstreams < 0) return LZMA_E_PARAM;
    if (lzma_params_check(p) != LZMA_OK) return fail(m, LZMA_E_PARAM, "invalid lzma_params");
    for (int i = 0; i < nstreams; i++)
        if (offs[i + 1] < offs[i]) return fail(m, LZMA_E_PARAM, "offsets not monotone");
    const int D = (int)m->ctxs.size();
    Deal deal(nstreams, D);
    std::vector<std::vector<uint8_t>> outs(D);
    std::vector<std::vector<uint64_t>> oofs(D);
    std::vector<int> rcs(D, LZMA_OK);
    std::vector<std::string> why(D);
    auto work = [&](int j) { guarded([&] {
        const std::vector<int>& idx = deal.idx[j];
        const int n = (int)idx.size();
        std::vector<uint64_t> lo(n + 1, 0);
        uint64_t cap = 1;
        for (int k = 0; k < n; k++) {
            const uint64_t len = offs[idx[k] + 1] - offs[idx[k]];
            lo[k + 1] = lo[k] + len;
            cap += lzma_enc_bound(len);
        }
        std::vector<uint8_t> buf(lo[n] + 1);   // the device's streams back to back
        for (int k = 0; k < n; k++) memcpy(buf.data() + lo[k], in + offs[idx[k]], lo[k + 1] - lo[k]);
        outs[j].resize(cap);
        oofs[j].assign(n + 1, 0);
        if (n) rcs[j] = lzma_enc_batch(m->ctxs[j], p, buf.data(), lo.data(), n, outs[j].data(), cap, oofs[j].data());
        if (rcs[j] != LZMA_OK) why[j] = lzma_last_error(m->ctxs[j]);
    }, rcs[j], why[j]); };
    std::vector<std::thread> th;
    for (int j = 1; j < D; j++) th.emplace_back(work, j);
    work(0);
    for (auto& t : th) t.join();
    for (int j = 0; j < D; j++)
        if (rcs[j] != LZMA_OK) return fail(m, rcs[j], "device " + std::to_string(m->devices[j]) + ": " + why[j]);
    out_offs[0] = 0;
    std::vector<size_t> pos(D, 0);
    for (int i = 0; i < nstreams; i++) {   // stream i is the (i / D)-th of device i % D
        const int j = i % D;
        const size_t k = pos[j]++;
        out_offs[i + 1] = out_offs[i] + (oofs[j][k + 1] - oofs[j][k]);
    }
    if (out_offs[nstreams] > out_cap) return fail(m, LZMA_E_OVERFLOW, "out_cap too small");
    std::fill(pos.begin(), pos.end(), 0);
    for (int i = 0; i < nstreams; i++) {
        const int j = i % D;
        const size_t k = pos[j]++;
        const uint64_t len = oofs[j][k + 1] - oofs[j][k];
        if (len) memcpy(out + out_offs[i], outs[j].data() + oofs[j][k], len);
    }
    return LZMA_OK;
}

int lzma_dec_batch_multi(lzma_mctx* m, const uint8_t props[5], const uint8_t* in, const uint64_t* in_offs,
                         int nstreams, const int64_t* out_sizes, uint8_t* out, const uint64_t* out_offs,
                         uint64_t* out_lens, int32_t* status) {
    if (!valid(m) || !props || !in_offs || !out_sizes || !out_offs || !out_lens || !status || nstreams < 0)
        return LZMA_E_PARAM;
    for (int i = 0; i < nstreams; i++)
        if (in_offs[i + 1] < in_offs[i] || out_offs[i + 1] < out_offs[i])
            return fail(m, LZMA_E_PARAM, "offsets not monotone");
    const int D = (int)m->ctxs.size();
    Deal deal(nstreams, D);
    std::vector<int> rcs(D, LZMA_OK);
    std::vector<std::string> why(D);
    // per device: its streams' output regions back to back, lengths and statuses; the
    // caller's arrays are written only after every device succeeded
    std::vector<std::vector<uint8_t>> dsts(D);
    std::vector<std::vector<uint64_t>> oos(D), lenss(D);
    std::vector<std::vector<int32_t>> sts(D);
    auto work = [&](int j) { guarded([&] {
        const std::vector<int>& idx = deal.idx[j];
        const int n = (int)idx.size();
        if (!n) return;
        std::vector<uint64_t> io(n + 1, 0);
        std::vector<uint64_t>& oo = oos[j];
        oo.assign(n + 1, 0);
        lenss[j].assign(n, 0);
        sts[j].assign(n, 0);
        std::vector<int64_t> sizes(n);
        for (int k = 0; k < n; k++) {
            const int i = idx[k];
            io[k + 1] = io[k] + (in_offs[i + 1] - in_offs[i]);
            oo[k + 1] = oo[k] + (out_offs[i + 1] - out_offs[i]);
            sizes[k] = out_sizes[i];
        }
        std::vector<uint8_t> src(io[n] + 1);
        dsts[j].resize(oo[n] + 1);
        for (int k = 0; k < n; k++) memcpy(src.data() + io[k], in + in_offs[idx[k]], io[k + 1] - io[k]);
        rcs[j] = lzma_dec_batch(m->ctxs[j], props, src.data(), io.data(), n, sizes.data(), dsts[j].data(), oo.data(),
                                lenss[j].data(), sts[j].data());
        if (rcs[j] != LZMA_OK) why[j] = lzma_last_error(m->ctxs[j]);
    }, rcs[j], why[j]); };
    std::vector<std::thread> th;
    for (int j = 1; j < D; j++) th.emplace_back(work, j);
    work(0);
    for (auto& t : th) t.join();
    for (int j = 0; j < D; j++)
        if (rcs[j] != LZMA_OK) return fail(m, rcs[j], "device " + std::to_string(m->devices[j]) + ": " + why[j]);
    for (int j = 0; j < D; j++) {
        const std::vector<int>& idx = deal.idx[j];
        for (size_t k = 0; k < idx.size(); k++) {
            const int i = idx[k];
            out_lens[i] = lenss[j][k];
            status[i] = sts[j][k];
            const uint64_t L = std::min<uint64_t>(lenss[j][k], oos[j][k + 1] - oos[j][k]);
            if (L) memcpy(out + out_offs[i], dsts[j].data() + oos[j][k], L);
        }
    }
    return LZMA_OK;
}

}  // extern "C"
