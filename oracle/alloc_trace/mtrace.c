/* oracle/alloc_trace/mtrace.c — TEST INFRASTRUCTURE ONLY.
 *
 * Linked into a trace build of the reference (oracle/Makefile: _ref/ref_COMPRESS_mtrace) to
 * log every heap call of a standalone COMPRESS run. The executable's malloc/free/calloc/realloc
 * interpose libc's (libstdc++'s operator new calls malloc through the PLT) and forward to
 * glibc's own __libc_* entry points, so the heap evolves exactly as in the untraced binary;
 * the logger itself never allocates (fixed stack buffer, write(2) to the fd named by
 * BMH_MTRACE_FD, default 2). One line per call:
 *   M <size> <addr>     malloc / operator new
 *   C <size> <addr>     calloc (size = nmemb * size)
 *   R <size> <old> <new> realloc
 *   F <addr>            free (non-null)
 * The reference's Huffman tie-break compares BTree* addresses (main.cpp:232,240,252), so the
 * order of the 24-byte allocations inside huffman() is what decides its tree bytes.
 */
#define _GNU_SOURCE
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <unistd.h>

extern void *__libc_malloc(size_t);
extern void __libc_free(void *);
extern void *__libc_calloc(size_t, size_t);
extern void *__libc_realloc(void *, size_t);

static int g_fd = -1;

static int out_fd(void)
{
    if (g_fd < 0) {
        const char *e = getenv("BMH_MTRACE_FD");
        g_fd = 2;
        if (e && *e) {
            int v = 0;
            for (; *e >= '0' && *e <= '9'; ++e) v = v * 10 + (*e - '0');
            g_fd = v;
        }
    }
    return g_fd;
}

static char *put_hex(char *p, uint64_t v)
{
    char t[17];
    int n = 0;
    do {
        t[n++] = "0123456789abcdef"[v & 15];
        v >>= 4;
    } while (v);
    *p++ = '0';
    *p++ = 'x';
    while (n) *p++ = t[--n];
    return p;
}

static char *put_dec(char *p, uint64_t v)
{
    char t[21];
    int n = 0;
    do {
        t[n++] = (char)('0' + v % 10);
        v /= 10;
    } while (v);
    while (n) *p++ = t[--n];
    return p;
}

static void emit(char op, size_t sz, const void *a, const void *b, int nargs)
{
    char buf[96], *p = buf;
    *p++ = op;
    if (op != 'F') {
        *p++ = ' ';
        p = put_dec(p, sz);
    }
    *p++ = ' ';
    p = put_hex(p, (uintptr_t)a);
    if (nargs > 1) {
        *p++ = ' ';
        p = put_hex(p, (uintptr_t)b);
    }
    *p++ = '\n';
    ssize_t r = write(out_fd(), buf, (size_t)(p - buf));
    (void)r;
}

void *malloc(size_t n)
{
    void *p = __libc_malloc(n);
    emit('M', n, p, 0, 1);
    return p;
}

void *calloc(size_t m, size_t n)
{
    void *p = __libc_calloc(m, n);
    emit('C', m * n, p, 0, 1);
    return p;
}

void *realloc(void *o, size_t n)
{
    void *p = __libc_realloc(o, n);
    emit('R', n, o, p, 2);
    return p;
}

void free(void *p)
{
    if (p) emit('F', 0, p, 0, 1);
    __libc_free(p);
}
