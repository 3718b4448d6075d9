// emu.h -- TEST INFRASTRUCTURE ONLY.
// A fiber-based SIMT emulator: every GPU lane of a block is a ucontext fiber;
// wave collectives (ballot, DPP, bpermute, readlane) and __syncthreads are
// rendezvous points resolved by a scheduler once every live lane of the wave
// (block) has arrived.  It lets tests run the product kernel source
// (vcf-compression_amd/csrc/*.hip) unmodified on the CPU, compiled with g++
// against the shim headers in this directory.  It is never part of the
// product library.
#pragma once
#include <ucontext.h>
#include <cstdint>
#include <functional>
#include <vector>

namespace emu {
struct dim3v {
    unsigned x = 1, y = 1, z = 1;
};
enum Op { OP_NONE = 0, OP_BALLOT, OP_DPP, OP_SHFL, OP_READFIRST, OP_WAVESYNC, OP_SYNCTHREADS };
struct Lane {
    ucontext_t ctx;
    dim3v tid;
    int linear = 0;
    bool done = false, waiting = false;
    int op = OP_NONE;
    uint64_t a = 0, b = 0, c = 0, out = 0;
};
struct State {
    dim3v grid, block, bid;
    std::vector<Lane> lanes;
    ucontext_t sched;
    Lane *cur = nullptr;
    std::function<void()> body;
    std::vector<std::vector<char>> stacks;
    uint64_t switches = 0;
};
extern State g;
uint64_t collective(int op, uint64_t a, uint64_t b, uint64_t c);
void launch(dim3v grid, dim3v block, std::function<void()> body);
inline unsigned lane() { return (unsigned)(g.cur->linear & 63); }
}  // namespace emu
