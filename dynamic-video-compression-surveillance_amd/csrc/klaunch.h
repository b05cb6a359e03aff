// klaunch.h — kernel launches that can also be recorded as graph nodes.
//
// Every FD launch function (fd_kernels.hip) launches through klaunch(). When
// a thread has set g_krec, klaunch() appends the launch — kernel, grid, block,
// dynamic LDS and the argument bytes as the kernel receives them — instead of
// launching, so fd_api.hip can build (and per call, re-parameterise) a HIP
// graph of one batch's launch sequence from the same code that launches it
// directly. Host only.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <tuple>
#include <type_traits>
#include <vector>

namespace dvc {

struct KNode {
    const void* f = nullptr;
    dim3 grid, block;
    uint32_t shm = 0;
    std::vector<uint8_t> args;   // parameter i at off[i], each at its own alignment
    std::vector<uint32_t> off;

    bool same_shape(const KNode& o) const
    {
        return f == o.f && grid.x == o.grid.x && grid.y == o.grid.y && grid.z == o.grid.z && block.x == o.block.x &&
               block.y == o.block.y && block.z == o.block.z && shm == o.shm && off == o.off &&
               args.size() == o.args.size();
    }
    // kernelParams for hipGraphAddKernelNode / hipGraphExecKernelNodeSetParams
    void params(std::vector<void*>& p) const
    {
        p.resize(off.size());
        for (size_t i = 0; i < off.size(); ++i) p[i] = const_cast<uint8_t*>(args.data()) + off[i];
    }
};

// non-null on this thread: klaunch() records into it instead of launching
extern thread_local std::vector<KNode>* g_krec;

template <typename V>
inline void knode_put(KNode& n, const V& v)
{
    size_t o = (n.args.size() + alignof(V) - 1) & ~(alignof(V) - 1);
    n.args.resize(o + sizeof(V));
    std::memcpy(n.args.data() + o, &v, sizeof(V));
    n.off.push_back((uint32_t)o);
}

template <typename... P, typename... A>
inline void klaunch(void (*k)(P...), dim3 grid, dim3 block, uint32_t shm, hipStream_t s, A&&... a)
{
    static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
    std::tuple<std::decay_t<P>...> t{static_cast<std::decay_t<P>>(a)...};
    if (g_krec) {
        KNode n;
        n.f = reinterpret_cast<const void*>(k);
        n.grid = grid;
        n.block = block;
        n.shm = shm;
        std::apply([&](const auto&... v) { (knode_put(n, v), ...); }, t);
        g_krec->push_back(std::move(n));
        return;
    }
    void* ptrs[sizeof...(P) > 0 ? sizeof...(P) : 1];
    size_t i = 0;
    std::apply([&](auto&... v) { ((ptrs[i++] = static_cast<void*>(&v)), ...); }, t);
    (void)hipLaunchKernel(reinterpret_cast<const void*>(k), grid, block, ptrs, shm, s);
}

}  // namespace dvc
