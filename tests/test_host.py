"""CPU: the product library's host side, without a GPU.

- libbmh.so loads and exports every function include/bmh.h declares;
- host-only stages (Huffman code book, record decode, container framing, MTF decode) agree
  with the reference's golden records;
- every device entry point fails loudly (BMH_ENODEV) when no gfx950 device is present —
  there is no CPU fallback in the product path.
"""
import json
import os
import re
import subprocess

import numpy as np
import pytest

import bmh
from oracle_ffi import GOLDEN, golden_calgary, golden_small

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "bmh.h")
CLI = os.path.join(REPO, "bwt-mtf-huffman-compressor_amd", "bin", "bmh")


def _declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = set(re.findall(r"\b(bmh_[a-z0-9_]+)\s*\(", txt))
    return sorted(n for n in names if not n.endswith("_t"))


def test_library_exports_every_declared_symbol():
    lib = bmh.lib()
    names = _declared()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", lib._name], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (bmh_\w+)", out))
    assert set(names) <= exported


def test_version_and_status_strings():
    assert bmh.lib().bmh_version().decode().startswith("bmh ")
    for st in range(7):
        assert bmh.lib().bmh_status_str(st)


def _hist(mtf: bytes):
    a = np.frombuffer(mtf, np.uint8)
    freq = np.bincount(a, minlength=256).astype(np.uint64)
    first = np.full(256, np.iinfo(np.uint64).max, np.uint64)
    idx = np.unique(a, return_index=True)
    first[idx[0]] = idx[1]
    return freq, first


def test_huffman_build_reproduces_golden_trees():
    """Host code book vs the reference's own tree bytes and payload sizes (App. B tie-break)."""
    for name, data, rec in list(golden_calgary()) + list(golden_small()):
        mtf = bmh.record_to_mtf(rec)
        freq, first = _hist(mtf)
        t = bmh.huffman_build(freq, first)
        tl = int.from_bytes(rec[16:24], "little")
        assert t.tree_len == tl, name
        assert t.tree_bytes == rec[24:24 + tl], name
        assert bmh.payload_bytes(t, freq) == len(rec) - 24 - tl, name


def test_decompress_golden_records():
    for name, data, rec in list(golden_calgary()) + list(golden_small()):
        assert bmh.decompress_bytes(rec) == data, name


def test_record_to_mtf_matches_oracle(oracle):
    for name, data, rec in golden_calgary():
        if len(data) > 200000:
            continue
        assert bmh.record_to_mtf(rec) == oracle.mtf(oracle.bwt(data)[1]), name


def test_container_framing():
    recs = [r for _, _, r in golden_small()]
    datas = [d for _, d, _ in golden_small()]
    bs = 1 << 20
    body = b"".join(recs)
    hdr = b"\xffBMHBLK1" + bs.to_bytes(8, "little") + len(recs).to_bytes(8, "little") + \
        sum(map(len, datas)).to_bytes(8, "little") + b"".join(len(r).to_bytes(8, "little") for r in recs)
    cont = hdr + body
    assert bmh.is_container(cont) and not bmh.is_container(recs[0])
    assert bmh.container_records(cont) == recs
    assert bmh.decompress_bytes(cont) == b"".join(datas)


@pytest.mark.parametrize("mutate", ["truncate", "bad_n", "bad_tree_len", "bad_primary"])
def test_corrupt_records_fail_loudly(mutate):
    _, data, rec = next(golden_calgary())
    r = bytearray(rec)
    if mutate == "truncate":
        r = r[:100]
    elif mutate == "bad_n":
        r[8:16] = (10 ** 12).to_bytes(8, "little")
    elif mutate == "bad_tree_len":
        r[16:24] = (10 ** 6).to_bytes(8, "little")
    else:
        r[0:8] = (len(data) + 5).to_bytes(8, "little")
    with pytest.raises(bmh.BmhError):
        bmh.decompress_bytes(bytes(r))


def test_metrics_line_matches_reference_stdout():
    gold = {e["file"]: e["stdout_tail"] for e in json.load(open(os.path.join(GOLDEN, "calgary_stdout.json")))}
    for name, data, rec in golden_calgary():
        hdr = 24 + int.from_bytes(rec[16:24], "little")
        line = bmh.metrics_line(name + ".bzap", len(data), len(rec), hdr) + "\n"
        assert line.endswith(gold[name]), name


@pytest.mark.skipif(bmh.lib().bmh_device_count() > 0, reason="a GPU is present")
def test_device_paths_fail_loudly_without_gpu():
    with pytest.raises(bmh.BmhError) as e:
        bmh.Context(0)
    assert e.value.status == 6  # BMH_ENODEV
    with pytest.raises(bmh.BmhError):
        bmh.bwt(b"banana")


@pytest.mark.skipif(not os.path.exists(CLI), reason="CLI not built")
def test_cli_host_modes(tmp_path):
    # the per-mode aliases behave like the reference's per-mode binaries (main.cpp:439-451)
    r = subprocess.run([CLI + "_compress", "only_one_arg"], capture_output=True, text=True)
    assert r.returncode == 1 and r.stdout == "Wrong arguments. Pass only input and output file as parameters"
    name, data, rec = next(golden_calgary())
    src = tmp_path / "bib.bzap"
    src.write_bytes(rec)
    out = tmp_path / "bib.out"
    # --host: libbmh's host C++ decoder (bmh decompress decodes on the GPU by default)
    r = subprocess.run([CLI, "decompress", str(src), str(out), "--host"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == data
    if bmh.lib().bmh_device_count() == 0:
        r = subprocess.run([CLI, "compress", str(out), str(tmp_path / "x.bzap")], capture_output=True, text=True)
        assert r.returncode != 0 and "device" in (r.stderr + r.stdout).lower()
        r = subprocess.run([CLI, "decompress", str(src), str(tmp_path / "y.out")], capture_output=True, text=True)
        assert r.returncode != 0 and "device" in (r.stderr + r.stdout).lower()
        assert not (tmp_path / "y.out").exists()


@pytest.mark.parametrize("nsym", [2, 12, 34, 38, 60])
def test_huffman_build_long_codes_matches_oracle(oracle, nsym):
    """bmh_huffman_build (host; huffman() tree, main.cpp:245-254) on Fibonacci frequencies,
    whose tree is a chain with codes up to nsym-1 bits (beyond 32 and up to 59), against the
    oracle's code lengths, codes and tree bytes, with leaves in a shuffled first-occurrence
    order."""
    f = [1, 1]
    while len(f) < nsym:
        f.append(f[-1] + f[-2])
    rng = np.random.default_rng(nsym)
    vals = rng.permutation(256)[:nsym]
    freq = np.zeros(256, np.uint64)
    first = np.full(256, np.iinfo(np.uint64).max, np.uint64)
    freq[vals] = f[:nsym]
    first[vals] = rng.permutation(nsym).astype(np.uint64) * 7
    t = bmh.huffman_build(freq, first)
    oln, ocode, otree = oracle.huffman_build(freq, first)
    ln = np.frombuffer(bytes(t.len), np.uint8)
    assert (ln == oln).all() and int(ln.max()) == nsym - 1
    code = np.ctypeslib.as_array(t.code)
    assert (code[oln > 0] == ocode[oln > 0]).all()
    assert t.tree_bytes == otree
    assert bmh.payload_bytes(t, freq) == max(1, (int((freq * ln.astype(np.uint64)).sum()) + 7) // 8)


ASAN_BIN = os.path.join(REPO, "bwt-mtf-huffman-compressor_amd", "bin", "host_asan")


def test_host_code_under_asan_ubsan():
    """SURVEY §5 (race detection / sanitizers): the host sources of libbmh (record decode,
    container framing, Huffman code books, status paths) built with ASan + UBSan
    (`make asan`; device code unsanitised) and driven by tests/asan/host_asan.cpp over golden
    records, every header truncation, edge-valued header fields, random byte flips and damaged
    container tables. Any overrun or UB aborts the driver."""
    pkg = os.path.join(REPO, "bwt-mtf-huffman-compressor_amd")
    b = subprocess.run(["make", "-C", pkg, "asan"], capture_output=True, text=True, timeout=900)
    assert b.returncode == 0, b.stdout[-2000:] + b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    names = ["bib", "paper1", "paper2", "progc", "progl", "progp", "trans", "obj1", "geo"]
    r = subprocess.run([ASAN_BIN, GOLDEN] + names, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failure(s)" in r.stdout


def test_compress_host_multi_rejects_bad_context_lists():
    """bmh_compress_host_multi drives each context from its own host thread: a context listed
    twice, or a null entry, is refused (BMH_EINVAL) before any device is touched."""
    import ctypes as C
    L = bmh.lib()
    data = np.frombuffer(b"banana" * 100, np.uint8)
    out = np.zeros(4096, np.uint8)
    olen = np.zeros(1, np.uint64)
    fake = C.c_void_p(0x1000)
    for lst in ([fake, fake], [fake, C.c_void_p(0)]):
        arr = (C.c_void_p * len(lst))(*lst)
        st = L.bmh_compress_host_multi(arr, len(lst), data.ctypes.data, data.size, 64, out.ctypes.data, out.size,
                                       olen.ctypes.data_as(bmh.PU64))
        assert st == bmh.BMH_EINVAL
        assert "context" in L.bmh_last_error().decode()


def _cgroup_cpus():
    """The CPU count this process may use, restated: affinity set, capped by the cgroup quota."""
    n = len(os.sched_getaffinity(0))
    q = None
    try:
        a, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if a != "max":
            q = -(-int(a) // int(per))
    except (OSError, ValueError):
        try:
            qa = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            pe = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if qa > 0 and pe > 0:
                q = -(-qa // pe)
        except (OSError, ValueError):
            q = None
    return max(1, min(n, q)) if q else n


def test_copy_thread_budget_follows_cpus_and_contexts():
    """the host-buffer path's staging copies are sized from the CPUs the process
    may use (affinity set capped by the cgroup quota), divided across the contexts streaming at
    once, instead of hardware_concurrency() per context. On the driver's boxes (16 CPUs granted of
    256) 8 contexts get 2 copy threads a site each, not 16 each."""
    L = bmh.lib()
    assert L.bmh_host_cpus() == _cgroup_cpus()
    assert L.bmh_copy_threads(8, 16) == 2
    assert L.bmh_copy_threads(1, 16) == 16
    assert L.bmh_copy_threads(8, 256) == 16
    assert L.bmh_copy_threads(16, 8) == 1
    assert L.bmh_copy_threads(3, 16) == 5
    assert L.bmh_copy_threads(0, 16) == 16  # no share given: one context
    assert L.bmh_copy_threads(1, 0) == min(16, _cgroup_cpus())
    # 8 contexts under a 16-CPU quota: at most 2 sites x 8 contexts x 2 threads = 32 copy threads
    assert 2 * 8 * L.bmh_copy_threads(8, 16) <= 2 * 16
