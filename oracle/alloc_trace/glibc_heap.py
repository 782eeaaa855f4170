"""oracle/alloc_trace/glibc_heap.py — TEST INFRASTRUCTURE ONLY.

A restatement of glibc 2.35's main-arena allocator (malloc/malloc.c: __libc_malloc, _int_malloc,
_int_free, malloc_consolidate, sysmalloc, systrim; x86-64 constants) — enough of it to replay the
heap calls of one standalone reference COMPRESS run and return the address of every block.
The reference's Huffman tie-break compares BTree* addresses (main.cpp:232,240,252), so the
order of the 24-byte blocks huffman() allocates is what decides its tree bytes below 64.6 KB.

Addresses are offsets from the start of the heap (the brk start, page aligned); blocks served
by mmap get addresses >= MMAP_BASE. Only the calls the reference makes are modelled (malloc,
free; no calloc / realloc / memalign), one thread, no arenas, no checks.

Validated call by call against traces of the real binary (oracle/alloc_trace/mtrace.c,
band_trace.py --validate).
"""
from __future__ import annotations

SIZE_SZ = 8
ALIGN = 16
MINSIZE = 32
PAGE = 4096
TCACHE_BINS = 64
TCACHE_COUNT = 7
MAX_FAST = 128                      # global_max_fast: (DEFAULT_MXFAST 128 + SIZE_SZ) & ~15
MIN_LARGE = 1024                    # in_smallbin_range: size < 64 * 16
CONSOLIDATE_AT = 65536              # FASTBIN_CONSOLIDATION_THRESHOLD
TOP_PAD = 128 * 1024                # DEFAULT_TOP_PAD
MMAP_THRESHOLD_MAX = 32 << 20       # DEFAULT_MMAP_THRESHOLD_MAX (64-bit)
MMAP_BASE = 1 << 44


def request2size(req: int) -> int:
    return max(MINSIZE, (req + SIZE_SZ + ALIGN - 1) & ~(ALIGN - 1))


def largebin_index(sz: int) -> int:
    if (sz >> 6) <= 48:
        return 48 + (sz >> 6)
    if (sz >> 9) <= 20:
        return 91 + (sz >> 9)
    if (sz >> 12) <= 10:
        return 110 + (sz >> 12)
    if (sz >> 15) <= 4:
        return 119 + (sz >> 15)
    if (sz >> 18) <= 2:
        return 124 + (sz >> 18)
    return 126


def bin_index(sz: int) -> int:
    return sz >> 4 if sz < MIN_LARGE else largebin_index(sz)


class Heap:
    """State: chunk map, top, tcache, fastbins, unsorted / small / large bins."""

    def __init__(self) -> None:
        self.size = {}          # chunk address -> chunk size (every chunk carved from the heap)
        self.free = set()       # chunks in unsorted / small / large bins (inuse bit clear)
        self.where = {}         # free chunk -> bin index (1 = unsorted)
        self.bins = {}          # bin index -> list, head (fd side) first
        self.tcache = [[] for _ in range(TCACHE_BINS)]   # LIFO: last element = head
        self.fast = [[] for _ in range(10)]              # LIFO: last element = head
        self.have_fast = False
        self.top = 0
        self.top_size = 0
        self.brk_end = 0
        self.last_remainder = None
        self.mmap_threshold = 128 * 1024
        self.trim_threshold = 128 * 1024
        self.mmapped = {}       # mem address -> chunk size
        self.mmap_next = MMAP_BASE
        self.tcache_ready = False

    # ---- bins
    def _bin(self, i: int) -> list:
        return self.bins.setdefault(i, [])

    def _unlink(self, p: int) -> None:
        i = self.where.pop(p)
        self._bin(i).remove(p)
        self.free.discard(p)
        if self.last_remainder == p:
            pass  # glibc keeps the stale pointer; it is only compared by identity

    def _to_unsorted(self, p: int) -> None:
        self._bin(1).insert(0, p)
        self.where[p] = 1
        self.free.add(p)

    def _place(self, p: int) -> None:
        """unsorted -> small bin (head) or large bin (size-sorted, glibc's insertion rule)."""
        sz = self.size[p]
        if sz < MIN_LARGE:
            i = sz >> 4
            self._bin(i).insert(0, p)
        else:
            i = largebin_index(sz)
            b = self._bin(i)
            if not b or sz < self.size[b[-1]]:
                b.append(p)
            else:
                k = 0
                # walk the size leaders from the largest down while sz < leader size
                while sz < self.size[b[k]]:
                    s = self.size[b[k]]
                    while k < len(b) and self.size[b[k]] == s:
                        k += 1
                if sz == self.size[b[k]]:
                    b.insert(k + 1, p)   # always the second position of its size
                else:
                    b.insert(k, p)
        self.where[p] = i
        self.free.add(p)

    # ---- top / system
    def _sysmalloc(self, nb: int) -> int:
        if nb >= self.mmap_threshold:
            sz = (nb + SIZE_SZ + PAGE - 1) & ~(PAGE - 1)
            mem = self.mmap_next + 16
            self.mmap_next += sz + PAGE
            self.mmapped[mem] = sz
            return mem
        size = nb + TOP_PAD + MINSIZE - self.top_size
        size = (size + PAGE - 1) & ~(PAGE - 1)
        self.brk_end += size
        self.top_size += size
        return self._from_top(nb)

    def _from_top(self, nb: int) -> int:
        p = self.top
        self.size[p] = nb
        self.top += nb
        self.top_size -= nb
        return p + 16

    def _split(self, p: int, nb: int, small_req: bool) -> int:
        sz = self.size[p]
        if sz - nb >= MINSIZE:
            r = p + nb
            self.size[p] = nb
            self.size[r] = sz - nb
            self._to_unsorted(r)
            if small_req:
                self.last_remainder = r
        return p + 16

    def _consolidate(self) -> None:
        self.have_fast = False
        for fb in self.fast:
            chain = list(reversed(fb))   # from the head, following fd
            fb.clear()
            for p in chain:
                self._coalesce_free(p)

    def _coalesce_free(self, p: int) -> int:
        """free-side merging of chunk p (not in any bin); returns the merged chunk's size."""
        sz = self.size[p]
        # previous chunk free? (only bin chunks have their inuse bit clear)
        prev = self._prev_free(p)
        if prev is not None:
            self._unlink(prev)
            del self.size[p]
            sz += self.size[prev]
            p = prev
            self.size[p] = sz
        nxt = p + sz
        if nxt == self.top:
            del self.size[p]
            self.top = p
            self.top_size += sz
            return self.top_size
        if nxt in self.free:
            self._unlink(nxt)
            sz += self.size.pop(nxt)
            self.size[p] = sz
        self._to_unsorted(p)
        return sz

    def _prev_free(self, p: int):
        for q in self.free:
            if q + self.size[q] == p:
                return q
        return None

    def _systrim(self) -> None:
        area = self.top_size - MINSIZE - 1
        if area <= TOP_PAD:
            return
        extra = (area - TOP_PAD) & ~(PAGE - 1)
        if extra > 0:
            self.top_size -= extra
            self.brk_end -= extra

    # ---- public
    def malloc(self, req: int) -> int:
        nb = request2size(req)
        if not self.tcache_ready:   # tcache_init: the per-thread struct is the heap's first chunk
            self.tcache_ready = True
            self._int_malloc(request2size(0x280))
        ti = (nb - MINSIZE) // ALIGN
        if ti < TCACHE_BINS and self.tcache[ti]:
            return self.tcache[ti].pop() + 16
        return self._int_malloc(nb)

    def _tcache_put(self, p: int) -> bool:
        ti = (self.size[p] - MINSIZE) // ALIGN
        if ti < TCACHE_BINS and len(self.tcache[ti]) < TCACHE_COUNT:
            self.tcache[ti].append(p)
            return True
        return False

    def _int_malloc(self, nb: int) -> int:
        ti = (nb - MINSIZE) // ALIGN
        tc_ok = ti < TCACHE_BINS
        small = nb < MIN_LARGE
        if nb <= MAX_FAST:
            fb = self.fast[(nb >> 4) - 2]
            if fb:
                v = fb.pop()
                while tc_ok and len(self.tcache[ti]) < TCACHE_COUNT and fb:
                    self.tcache[ti].append(fb.pop())
                return v + 16
        if small:
            b = self._bin(nb >> 4)
            if b:
                v = b.pop()
                del self.where[v]
                self.free.discard(v)
                while tc_ok and len(self.tcache[ti]) < TCACHE_COUNT and b:
                    t = b.pop()
                    del self.where[t]
                    self.free.discard(t)
                    self.tcache[ti].append(t)
                return v + 16
        elif self.have_fast:
            self._consolidate()
        while True:
            ret_cached = False
            ub = self._bin(1)
            iters = 0
            while ub:
                v = ub[-1]
                sz = self.size[v]
                if small and len(ub) == 1 and v == self.last_remainder and sz > nb + MINSIZE:
                    ub.pop()
                    del self.where[v]
                    self.free.discard(v)
                    return self._split(v, nb, True)
                ub.pop()
                del self.where[v]
                self.free.discard(v)
                if sz == nb:
                    if tc_ok and len(self.tcache[ti]) < TCACHE_COUNT:
                        self.tcache[ti].append(v)
                        ret_cached = True
                        continue
                    return v + 16
                self._place(v)
                iters += 1
                if iters >= 10000:
                    break
            if ret_cached:
                return self.tcache[ti].pop() + 16
            if not small:
                b = self._bin(largebin_index(nb))
                if b and self.size[b[0]] >= nb:
                    # the smallest size group whose size >= nb, its second member if it has one
                    k = len(b) - 1
                    while self.size[b[k]] < nb:
                        k -= 1
                    s = self.size[b[k]]
                    while k > 0 and self.size[b[k - 1]] == s:
                        k -= 1
                    if k + 1 < len(b) and self.size[b[k + 1]] == s:
                        k += 1
                    v = b.pop(k)
                    del self.where[v]
                    self.free.discard(v)
                    return self._split(v, nb, False)
            for i in range(bin_index(nb) + 1, 128):
                b = self.bins.get(i)
                if b:
                    v = b.pop()
                    del self.where[v]
                    self.free.discard(v)
                    return self._split(v, nb, small)
            if self.top_size >= nb + MINSIZE:
                return self._from_top(nb)
            if self.have_fast:
                self._consolidate()
                continue
            return self._sysmalloc(nb)

    def free_(self, mem: int) -> None:
        if mem in self.mmapped:
            sz = self.mmapped.pop(mem)
            if self.mmap_threshold < sz <= MMAP_THRESHOLD_MAX:
                self.mmap_threshold = sz
                self.trim_threshold = 2 * sz
            return
        p = mem - 16
        if self._tcache_put(p):
            return
        if self.size[p] <= MAX_FAST:
            self.fast[(self.size[p] >> 4) - 2].append(p)
            self.have_fast = True
            return
        sz = self._coalesce_free(p)
        if sz >= CONSOLIDATE_AT:
            if self.have_fast:
                self._consolidate()
            if self.top_size >= self.trim_threshold:
                self._systrim()
