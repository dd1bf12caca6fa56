// TEST INFRASTRUCTURE ONLY -- CPU stand-ins for the hipcub primitives the
// runtime uses (stable radix sort by a bit range, whole or per segment; flagged select), for the
// SIMT emulation build in tests/simt. Not part of the product build.
#pragma once
#include <algorithm>
#include <cstdint>
#include <numeric>
#include <vector>

namespace hipcub {
template <typename T>
struct CountingInputIterator {
    T v;
    explicit CountingInputIterator(T x) : v(x) {}
    T operator[](size_t i) const { return v + (T)i; }
};
struct DeviceRadixSort {
    template <typename K, typename V>
    static int sort(void* tmp, size_t& bytes, const K* kin, K* kout, const V* vin, V* vout, int n, int b0, int b1, bool desc) {
        if (!tmp) { bytes = 16; return 0; }
        auto key = [&](K k) -> uint64_t {
            uint64_t x = (uint64_t)k >> b0;
            int w = b1 - b0;
            return w >= 64 ? x : (x & ((1ull << w) - 1));
        };
        std::vector<int> idx(n);
        std::iota(idx.begin(), idx.end(), 0);
        std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) {
            return desc ? key(kin[a]) > key(kin[b]) : key(kin[a]) < key(kin[b]);
        });
        std::vector<K> ko(n);
        std::vector<V> vo(n);
        for (int i = 0; i < n; i++) { ko[i] = kin[idx[i]]; vo[i] = vin[idx[i]]; }
        std::copy(ko.begin(), ko.end(), kout);
        std::copy(vo.begin(), vo.end(), vout);
        return 0;
    }
    template <typename K, typename V, typename S>
    static int SortPairs(void* tmp, size_t& bytes, const K* kin, K* kout, const V* vin, V* vout, int n, int b0, int b1, S) {
        return sort(tmp, bytes, kin, kout, vin, vout, n, b0, b1, false);
    }
    template <typename K, typename V, typename S>
    static int SortPairsDescending(void* tmp, size_t& bytes, const K* kin, K* kout, const V* vin, V* vout, int n, int b0, int b1, S) {
        return sort(tmp, bytes, kin, kout, vin, vout, n, b0, b1, true);
    }
};
struct DeviceSegmentedRadixSort {
    template <typename K, typename V, typename O, typename S>
    static int SortPairs(void* tmp, size_t& bytes, const K* kin, K* kout, const V* vin, V* vout, int n, int nseg, O begin,
                         O end, int b0, int b1, S s) {
        if (!tmp) { bytes = 16; return 0; }
        std::copy(kin, kin + n, kout);   // items outside every segment keep their place
        std::copy(vin, vin + n, vout);
        for (int g = 0; g < nseg; g++) {
            const size_t lo = (size_t)begin[g], hi = (size_t)end[g];
            if (hi > lo) DeviceRadixSort::sort(tmp, bytes, kin + lo, kout + lo, vin + lo, vout + lo, (int)(hi - lo), b0, b1, false);
        }
        (void)s;
        return 0;
    }
};
struct DeviceSelect {
    template <typename It, typename F, typename O, typename C, typename S>
    static int Flagged(void* tmp, size_t& bytes, It in, const F* flags, O* out, C* num, int n, S) {
        if (!tmp) { bytes = 16; return 0; }
        C k = 0;
        for (int i = 0; i < n; i++)
            if (flags[i]) out[k++] = in[i];
        *num = k;
        return 0;
    }
};
}  // namespace hipcub
