// emu.cpp -- TEST INFRASTRUCTURE ONLY: scheduler of the fiber SIMT emulator.
#include "emu.h"
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace emu {
State g;
static const size_t STACK = 256 * 1024;

uint64_t collective(int op, uint64_t a, uint64_t b, uint64_t c) {
    Lane *l = g.cur;
    l->op = op; l->a = a; l->b = b; l->c = c; l->waiting = true;
    g.switches++;
    swapcontext(&l->ctx, &g.sched);
    return l->out;
}

static void entry() {
    g.body();
    g.cur->done = true;
    swapcontext(&g.cur->ctx, &g.sched);
}

static int dpp_src(int ctrl, int i) {
    int r = i & 15;
    if (ctrl >= 0x111 && ctrl <= 0x11F) { int n = ctrl - 0x110; return r >= n ? i - n : -1; }
    if (ctrl >= 0x101 && ctrl <= 0x10F) { int n = ctrl - 0x100; return r + n < 16 ? i + n : -1; }
    if (ctrl == 0x138) return i >= 1 ? i - 1 : -1;   // wave_shr:1
    if (ctrl == 0x130) return i <= 62 ? i + 1 : -1;  // wave_shl:1
    if (ctrl == 0x142) return i >= 16 ? (i & ~15) - 1 : -1;  // row_bcast:15
    if (ctrl == 0x143) return i >= 32 ? 31 : -1;     // row_bcast:31
    fprintf(stderr, "emu: unsupported dpp ctrl 0x%x\n", ctrl);
    abort();
}

static void resolve_wave(int w, int n) {
    int lo = w * 64, hi = lo + 64 < n ? lo + 64 : n;
    int op = -1;
    for (int i = lo; i < hi; i++) {
        Lane &L = g.lanes[i];
        if (L.done) continue;
        if (op < 0) op = L.op;
        if (L.op != op) { fprintf(stderr, "emu: divergent collectives in wave %d (%d vs %d)\n", w, op, L.op); abort(); }
    }
    uint64_t mask = 0;
    for (int i = lo; i < hi; i++) if (!g.lanes[i].done) mask |= 1ull << (i - lo);
    switch (op) {
    case OP_BALLOT: {
        uint64_t m = 0;
        for (int i = lo; i < hi; i++) if (!g.lanes[i].done && g.lanes[i].a) m |= 1ull << (i - lo);
        for (int i = lo; i < hi; i++) g.lanes[i].out = m;
        break;
    }
    case OP_DPP: {
        uint64_t res[64];
        for (int i = lo; i < hi; i++) {
            Lane &L = g.lanes[i];
            if (L.done) continue;
            int ctrl = (int)(L.c & 0xFFFF), rm = (int)((L.c >> 16) & 0xF), bm = (int)((L.c >> 20) & 0xF);
            int bc = (int)((L.c >> 24) & 1);
            int li = i - lo, row = li >> 4, bank = (li & 15) >> 2;
            if (!((rm >> row) & 1) || !((bm >> bank) & 1)) { res[li] = L.a; continue; }
            int s = dpp_src(ctrl, li);
            if (s < 0 || lo + s >= hi || g.lanes[lo + s].done) res[li] = bc ? 0 : L.a;
            else res[li] = g.lanes[lo + s].b;
        }
        for (int i = lo; i < hi; i++) if (!g.lanes[i].done) g.lanes[i].out = res[i - lo] & 0xFFFFFFFFull;
        break;
    }
    case OP_SHFL: {
        uint64_t res[64];
        for (int i = lo; i < hi; i++) {
            if (g.lanes[i].done) continue;
            int s = (int)(g.lanes[i].b & 63);
            res[i - lo] = (lo + s < hi && !g.lanes[lo + s].done) ? g.lanes[lo + s].a : 0;
        }
        for (int i = lo; i < hi; i++) if (!g.lanes[i].done) g.lanes[i].out = res[i - lo];
        break;
    }
    case OP_READFIRST: {
        int f = lo + __builtin_ctzll(mask);
        for (int i = lo; i < hi; i++) g.lanes[i].out = g.lanes[f].a;
        break;
    }
    case OP_WAVESYNC:
        break;
    default:
        fprintf(stderr, "emu: bad op %d\n", op);
        abort();
    }
    for (int i = lo; i < hi; i++) g.lanes[i].waiting = false;
}

static void run_block() {
    int n = (int)(g.block.x * g.block.y * g.block.z);
    g.lanes.assign(n, Lane());
    if ((int)g.stacks.size() < n) g.stacks.resize(n);
    for (int i = 0; i < n; i++) {
        Lane &L = g.lanes[i];
        L.linear = i;
        L.tid.x = i % g.block.x;
        L.tid.y = (i / g.block.x) % g.block.y;
        L.tid.z = i / (g.block.x * g.block.y);
        if (g.stacks[i].size() < STACK) g.stacks[i].resize(STACK);
        getcontext(&L.ctx);
        L.ctx.uc_stack.ss_sp = g.stacks[i].data();
        L.ctx.uc_stack.ss_size = STACK;
        L.ctx.uc_link = nullptr;
        makecontext(&L.ctx, entry, 0);
    }
    int nw = (n + 63) / 64;
    for (;;) {
        for (int i = 0; i < n; i++) {
            Lane &L = g.lanes[i];
            if (L.done || L.waiting) continue;
            g.cur = &L;
            g.switches++;
            swapcontext(&g.sched, &L.ctx);
        }
        bool all_done = true, any_sync = false;
        for (int i = 0; i < n; i++) {
            if (!g.lanes[i].done) { all_done = false; if (g.lanes[i].op == OP_SYNCTHREADS) any_sync = true; }
        }
        if (all_done) break;
        bool released = false;
        if (any_sync) {
            bool all = true;
            for (int i = 0; i < n; i++) if (!g.lanes[i].done && g.lanes[i].op != OP_SYNCTHREADS) all = false;
            if (all) {
                for (int i = 0; i < n; i++) g.lanes[i].waiting = false;
                released = true;
            }
        }
        if (!released) {
            for (int w = 0; w < nw; w++) {
                int lo = w * 64, hi = lo + 64 < n ? lo + 64 : n;
                bool any = false, sync = false;
                for (int i = lo; i < hi; i++) if (!g.lanes[i].done) { any = true; if (g.lanes[i].op == OP_SYNCTHREADS) sync = true; }
                if (!any || sync) continue;
                resolve_wave(w, n);
                released = true;
            }
        }
        if (!released) { fprintf(stderr, "emu: deadlock (block %u)\n", g.bid.x); abort(); }
    }
}

void launch(dim3v grid, dim3v block, std::function<void()> body) {
    g.grid = grid; g.block = block; g.body = std::move(body);
    for (unsigned z = 0; z < grid.z; z++)
        for (unsigned y = 0; y < grid.y; y++)
            for (unsigned x = 0; x < grid.x; x++) {
                g.bid.x = x; g.bid.y = y; g.bid.z = z;
                run_block();
            }
}
}  // namespace emu
