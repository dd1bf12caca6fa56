// TEST INFRASTRUCTURE ONLY -- CPU SIMT emulation of the small HIP subset used
// by lzma-java_amd/csrc, so the exact kernel sources can be compiled with g++
// and run under AddressSanitizer/UBSan on a machine without a GPU (debugging
// aid and CPU-side check of kernel logic). Never part of the product build:
// this directory is only on the include path of tests/simt/Makefile.
//
// Model: a launch runs its blocks one after another; each block runs
// blockDim.x OS threads (one per lane). __syncthreads, __shfl*, __ballot are
// block barriers, so kernels must call them in uniform control flow -- the
// same requirement real wavefronts impose on shuffles.
#pragma once
#include <pthread.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <barrier>
#include <chrono>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#define __global__
#define __device__
#define __host__
#define __constant__
#define __shared__
#define __forceinline__ inline
#define __launch_bounds__(...)

typedef int hipError_t;
enum { hipSuccess = 0, hipErrorMemoryAllocation = 2 };
typedef struct ihipStream_t* hipStream_t;
typedef struct ihipEvent_t* hipEvent_t;
enum hipMemcpyKind { hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice, hipMemcpyHostToHost };
enum hipDeviceAttribute_t { hipDeviceAttributeMultiprocessorCount = 1 };
enum hipFuncAttribute { hipFuncAttributeMaxDynamicSharedMemorySize = 1 };

struct dim3 {
    unsigned x, y, z;
    constexpr dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};

namespace hipemu {
// ---- fibers: every lane of a block is a user-space fiber on ONE OS thread;
// a collective (__syncthreads/__shfl/__ballot) yields to the block scheduler,
// which resumes every lane once per barrier round.
extern "C" void hipemu_swap(void** save_sp, void* new_sp);
asm(R"(
.text
.weak hipemu_swap
.type hipemu_swap,@function
hipemu_swap:
    pushq %rbp
    pushq %rbx
    pushq %r12
    pushq %r13
    pushq %r14
    pushq %r15
    movq %rsp, (%rdi)
    movq %rsi, %rsp
    popq %r15
    popq %r14
    popq %r13
    popq %r12
    popq %rbx
    popq %rbp
    ret
.size hipemu_swap, .-hipemu_swap
)");

#if defined(__SANITIZE_ADDRESS__)
extern "C" void __sanitizer_start_switch_fiber(void** fake_stack_save, const void* bottom, size_t size);
extern "C" void __sanitizer_finish_switch_fiber(void* fake_stack_save, const void** bottom_old, size_t* size_old);
#define HIPEMU_START(save, b, s) __sanitizer_start_switch_fiber(save, b, s)
#define HIPEMU_FINISH(save, bo, so) __sanitizer_finish_switch_fiber(save, bo, so)
#else
#define HIPEMU_START(save, b, s) ((void)0)
#define HIPEMU_FINISH(save, bo, so) ((void)0)
#endif

struct Fiber {
    void* sp = nullptr;
    char* stack = nullptr;
    size_t ssize = 0;
    bool done = false;
    dim3 tid;
    void* fake = nullptr;
};
struct Sched {
    void* main_sp = nullptr;
    const void* main_bottom = nullptr;
    size_t main_size = 0;
    void* main_fake = nullptr;
    Fiber* cur = nullptr;
    const std::function<void()>* body = nullptr;
    uint64_t xch[1024];
};
inline thread_local Sched g_sched;
inline thread_local dim3 t_bid, g_bdim, g_gdim;
inline thread_local dim3 g_dummy_tid;

[[noreturn]] inline void fiber_entry() {
    Sched& s = g_sched;
    HIPEMU_FINISH(nullptr, &s.main_bottom, &s.main_size);
    (*s.body)();
    s.cur->done = true;
    HIPEMU_START(nullptr, s.main_bottom, s.main_size);
    void* dummy;
    hipemu_swap(&dummy, s.main_sp);
    __builtin_unreachable();
}
inline void resume(Fiber* f) {
    Sched& s = g_sched;
    s.cur = f;
    HIPEMU_START(&s.main_fake, f->stack, f->ssize);
    hipemu_swap(&s.main_sp, f->sp);
    HIPEMU_FINISH(s.main_fake, nullptr, nullptr);
}
inline void yield() {   // called on a fiber: back to the scheduler
    Sched& s = g_sched;
    Fiber* f = s.cur;
    HIPEMU_START(&f->fake, s.main_bottom, s.main_size);
    hipemu_swap(&f->sp, s.main_sp);
    HIPEMU_FINISH(f->fake, &s.main_bottom, &s.main_size);
}
inline void barrier() { yield(); }

// one emulated kernel at a time process-wide: the LDS backing store (smem) is
// shared, so host threads driving different emulated devices take turns
inline std::mutex g_launch_mu;
inline void launch(const std::function<void()>& body, dim3 grid, dim3 block) {
    std::lock_guard<std::mutex> lk(g_launch_mu);
    const unsigned nt = block.x;
    g_bdim = block;
    g_gdim = grid;
    const size_t SS = 512 * 1024;
    std::vector<Fiber> fibers(nt);
    for (auto& f : fibers) { f.stack = (char*)aligned_alloc(64, SS); f.ssize = SS; }
    g_sched.body = &body;
    static const bool trace = getenv("HIPEMU_TRACE") != nullptr;
    if (trace) fprintf(stderr, "hip-emu: launch grid %u block %u\n", grid.x, nt);
    for (unsigned b = 0; b < grid.x; b++) {
        if (trace) fprintf(stderr, "hip-emu:   block %u\n", b);
        uint64_t rounds = 0;
        t_bid = dim3(b, 0, 0);
        for (unsigned t = 0; t < nt; t++) {
            Fiber& f = fibers[t];
            f.done = false;
            f.tid = dim3(t, 0, 0);
            // initial frame: 6 callee-saved registers, then the entry as return address
            uintptr_t top = ((uintptr_t)(f.stack + SS) & ~(uintptr_t)15) - 8;
            void** sp = (void**)top;
            *--sp = (void*)&fiber_entry;
            for (int k = 0; k < 6; k++) *--sp = nullptr;
            f.sp = sp;
        }
        for (;;) {   // one barrier round per iteration
            if (trace && (++rounds % 100000) == 0) fprintf(stderr, "hip-emu:     %llu barrier rounds\n", (unsigned long long)rounds);
            unsigned done = 0;
            for (unsigned t = 0; t < nt; t++) {
                if (!fibers[t].done) resume(&fibers[t]);
                done += fibers[t].done;
            }
            if (done == nt) break;
            if (done != 0) { fprintf(stderr, "hip-emu: divergent barrier (%u of %u lanes returned)\n", done, nt); abort(); }
        }
    }
    for (auto& f : fibers) free(f.stack);
}
}  // namespace hipemu

#define threadIdx (::hipemu::g_sched.cur ? ::hipemu::g_sched.cur->tid : ::hipemu::g_dummy_tid)
#define blockIdx (::hipemu::t_bid)
#define blockDim (::hipemu::g_bdim)
#define gridDim (::hipemu::g_gdim)

#define hipLaunchKernelGGL(K, G, B, S, ST, ...) ::hipemu::launch([&]() { K(__VA_ARGS__); }, dim3(G), dim3(B))

inline void __syncthreads() { ::hipemu::barrier(); }

template <typename T>
inline T __shfl(T v, int src, int width = 64) {
    auto& s = ::hipemu::g_sched;
    unsigned lane = threadIdx.x;
    uint64_t slot = 0;
    memcpy(&slot, &v, sizeof(T));
    s.xch[lane] = slot;
    ::hipemu::barrier();
    uint64_t r = s.xch[(lane & ~63u) + ((unsigned)src & 63u)];
    ::hipemu::barrier();
    T out;
    memcpy(&out, &r, sizeof(T));
    return out;
}
template <typename T>
inline T __shfl_up(T v, unsigned delta, int width = 64) {
    const unsigned l = threadIdx.x & 63u;
    return __shfl(v, (int)(l >= delta ? l - delta : l), width);
}
template <typename T>
inline T __shfl_xor(T v, int mask, int width = 64) {
    return __shfl(v, (int)((threadIdx.x & 63u) ^ (unsigned)mask), width);
}
inline unsigned long long __ballot(int pred) {
    auto& s = ::hipemu::g_sched;
    unsigned lane = threadIdx.x;
    s.xch[lane] = pred ? 1 : 0;
    ::hipemu::barrier();
    unsigned long long m = 0;
    unsigned base = lane & ~63u;
    for (unsigned i = 0; i < 64 && base + i < blockDim.x; i++)
        if (s.xch[base + i]) m |= 1ull << i;
    ::hipemu::barrier();
    return m;
}
// rc.hip uses the raw ballot only as a wave-uniform "any lane" skip around code that is a
// no-op for lanes whose predicate is false, so the lane's own predicate is exact here (and
// needs no barrier: rc.hip lanes leave their loops at different times)
inline unsigned long long __builtin_amdgcn_ballot_w64(bool p) { return p ? 1ull : 0ull; }
// wave barrier: a block barrier here (the emulated lanes of a wave are not in lockstep)
#define __builtin_amdgcn_wave_barrier() ::hipemu::barrier()
// mbcnt: set bits of the mask below this lane's index within its 64-lane group
inline uint32_t __builtin_amdgcn_mbcnt_lo(uint32_t m, uint32_t acc) {
    const unsigned l = threadIdx.x & 63u;
    return acc + (uint32_t)__builtin_popcount(l >= 32 ? m : (m & ((1u << l) - 1u)));
}
inline uint32_t __builtin_amdgcn_mbcnt_hi(uint32_t m, uint32_t acc) {
    const unsigned l = threadIdx.x & 63u;
    return acc + (uint32_t)(l < 32 ? 0 : __builtin_popcount(m & (l == 32 ? 0u : ((1u << (l - 32)) - 1u))));
}
inline unsigned atomicAdd(unsigned* p, unsigned v);
#define __builtin_amdgcn_fence(order, scope) __atomic_signal_fence(__ATOMIC_SEQ_CST)
// wave width 1: the first active lane is the only lane
inline int __builtin_amdgcn_readfirstlane(int v) { return v; }
#ifdef LZG_PROF   // the encoder's phase profile: counters only (no clock in the emulation)
inline uint64_t __builtin_amdgcn_s_memtime() { return 0; }
inline uint64_t __builtin_amdgcn_s_memrealtime() { return 0; }
inline unsigned __builtin_amdgcn_s_getreg(int) { return 0; }
#endif
inline int __builtin_amdgcn_readlane(int v, int) { return v; }
#define __builtin_nontemporal_load(p) (*(p))
#define __builtin_nontemporal_store(v, p) (*(p) = (v))
struct __amdgpu_buffer_rsrc_t { uint8_t* base; uint32_t bytes; };
inline __amdgpu_buffer_rsrc_t __builtin_amdgcn_make_buffer_rsrc(void* p, int, uint32_t bytes, uint32_t) {
    return __amdgpu_buffer_rsrc_t{(uint8_t*)p, bytes};
}
inline uint32_t __builtin_amdgcn_raw_buffer_load_b32(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t soff, int) {
    if ((uint64_t)off + soff + 4 > r.bytes) { fprintf(stderr, "hip-emu: buffer load out of range\n"); abort(); }
    uint32_t v; memcpy(&v, r.base + off + soff, 4); return v;
}
inline void __builtin_amdgcn_raw_buffer_store_b32(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t soff, int) {
    if (off + soff + 4 > r.bytes) { fprintf(stderr, "hip-emu: buffer store out of range\n"); abort(); }
    memcpy(r.base + off + soff, &v, 4);
}
inline uint8_t __builtin_amdgcn_raw_buffer_load_b8(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t soff, int) {
    uint64_t o = (uint64_t)off + soff;
    return o < r.bytes ? r.base[o] : 0;   // hardware range check: out of range reads 0
}
#define __HIP_MEMORY_SCOPE_SYSTEM 0
#define __hip_atomic_store(p, v, order, scope) (*(p) = (v))
enum { hipHostMallocDefault = 0, hipHostMallocMapped = 2, hipHostMallocCoherent = 0x40000000 };
enum { hipEventDisableTiming = 2 };
inline hipError_t hipHostMalloc(void** p, size_t n, unsigned) { *p = malloc(n); return *p ? hipSuccess : hipErrorMemoryAllocation; }
inline hipError_t hipHostFree(void* p) { free(p); return hipSuccess; }
inline hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned) { *d = h; return hipSuccess; }
inline int __ffsll(long long x) { return __builtin_ffsll(x); }
inline int __clz(int x) { return __builtin_clz((unsigned)x); }
inline unsigned atomicAdd(unsigned* p, unsigned v) { unsigned o = *p; *p = o + v; return o; }
inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) { unsigned long long o = *p; *p = o + v; return o; }

// ---- runtime API: device memory is host memory
inline hipError_t hipGetDeviceCount(int* n) {   // HIPEMU_DEVICES emulated devices (default 1)
    const char* e = getenv("HIPEMU_DEVICES");
    *n = e ? atoi(e) : 1;
    return hipSuccess;
}
inline hipError_t hipSetDevice(int d) { int n = 0; hipGetDeviceCount(&n); return d >= 0 && d < n ? hipSuccess : 101; }
inline hipError_t hipGetDevice(int* d) { *d = 0; return hipSuccess; }
inline hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t, int) { *v = 2; return hipSuccess; }
inline hipError_t hipFuncSetAttribute(const void*, hipFuncAttribute, int) { return hipSuccess; }
template <typename T>
inline hipError_t hipMalloc(T** p, size_t n) {
    void* q = malloc(n ? n : 1);
    if (!q) return hipErrorMemoryAllocation;
    memset(q, 0xA5, n);   // poison: uninitialised device memory is not zero on a GPU either
    *p = (T*)q;
    return hipSuccess;
}
inline hipError_t hipFree(void* p) { free(p); return hipSuccess; }
inline hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) { if (n) memmove(d, s, n); return hipSuccess; }
inline hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind k, hipStream_t = nullptr) { return hipMemcpy(d, s, n, k); }
inline hipError_t hipMemset(void* d, int v, size_t n) { memset(d, v, n); return hipSuccess; }
inline hipError_t hipMemsetAsync(void* d, int v, size_t n, hipStream_t = nullptr) { return hipMemset(d, v, n); }
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
enum { hipStreamDefault = 0, hipStreamNonBlocking = 1 };
inline hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) {   // every stream is the one serial "device"
    *s = (hipStream_t) new char(0);
    return hipSuccess;
}
inline hipError_t hipStreamDestroy(hipStream_t s) { delete (char*)s; return hipSuccess; }
inline hipError_t hipDeviceSynchronize() { return hipSuccess; }
inline hipError_t hipGetLastError() { return hipSuccess; }
inline const char* hipGetErrorString(hipError_t) { return "hip-emu"; }
inline hipError_t hipEventCreate(hipEvent_t* e) { *e = (hipEvent_t) new double(0); return hipSuccess; }
inline hipError_t hipEventDestroy(hipEvent_t e) { delete (double*)e; return hipSuccess; }
inline hipError_t hipEventRecord(hipEvent_t e, hipStream_t = nullptr) {
    *(double*)e = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    return hipSuccess;
}
inline hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { return hipEventCreate(e); }
inline hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }   // one serial "device"
inline hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b) { *ms = (float)(*(double*)b - *(double*)a); return hipSuccess; }
