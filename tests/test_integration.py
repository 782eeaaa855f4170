"""The reference-side binding (integration/compress_bmh.cpp): the reference's compress() and
decompress() (main.cpp:300-345) rewritten against include/bmh.h, compiled against the
reference's own io_utilities.h (read_bytes' tuple form, write_bytes with its raw defaults) and
its 3-argument print_metrics (main.cpp:294-298), linked with libbmh.so.

CPU (needs /root/reference, i.e. the build container): the file compiles and links as written;
the wrong-argument contract of main.cpp:440-443 holds; compress() and decompress() both fail
loudly without a GPU (decompress() decodes on the GPU since round 6).
GPU: the binary built here (integration/_build, travels with the snapshot) compresses every
Calgary file to the reference's record and prints the reference's stdout line, and its
decompress() decodes every golden Calgary record on the GPU back to the file."""
import json
import os
import shutil
import subprocess

import pytest

from oracle_ffi import CALGARY, GOLDEN, golden_calgary

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = "/root/reference"
BUILT = os.path.join(REPO, "integration", "_build", "bmh_ref_compress")
LIB = os.path.join(REPO, "bwt-mtf-huffman-compressor_amd", "lib", "libbmh.so")


def _build(tmp_path) -> str:
    src = os.path.join(REPO, "integration")
    obj = tmp_path / "compress_bmh.o"
    exe = tmp_path / "bmh_ref_compress"
    subprocess.run(["g++", "-std=c++2b", "-O1", "-Wall", "-Werror", "-Wno-sign-compare", "-include", "climits",
                    "-I", REF_DIR, "-I", os.path.join(REPO, "include"), "-c", os.path.join(src, "compress_bmh.cpp"),
                    "-o", str(obj)], check=True, capture_output=True, text=True)
    libdir = os.path.dirname(LIB)
    subprocess.run(["g++", "-std=c++2b", "-O1", os.path.join(src, "driver.cpp"), str(obj), "-o", str(exe),
                    "-L" + libdir, "-lbmh", "-Wl,-rpath," + libdir, "-Wl,-rpath,/opt/rocm/lib"],
                   check=True, capture_output=True, text=True)
    os.symlink(exe, tmp_path / "bmh_ref_decompress")
    return str(exe)


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_DIR, "io_utilities.h")),
                    reason="the reference's headers are only in the build container")
def test_binding_compiles_against_reference_and_fails_loudly_without_gpu(tmp_path):
    exe = _build(tmp_path)
    dec = str(tmp_path / "bmh_ref_decompress")
    r = subprocess.run([exe, "only_one_arg"], capture_output=True, text=True)
    assert r.returncode == 1 and r.stdout == "Wrong arguments. Pass only input and output file as parameters"
    import torch
    if not torch.cuda.is_available():  # no CPU fallback: compress() and decompress() fail loudly
        name, data, rec = next(golden_calgary())
        (tmp_path / "bib").write_bytes(data)
        r = subprocess.run([exe, "bib", "fresh.bzap"], cwd=tmp_path, capture_output=True, text=True)
        assert r.returncode == 2 and "libbmh:" in r.stderr
        assert not (tmp_path / "fresh.bzap").exists()
        (tmp_path / "bib.bzap").write_bytes(rec)
        r = subprocess.run([dec, "bib.bzap", "bib.decoded"], cwd=tmp_path, capture_output=True, text=True)
        assert r.returncode == 2 and "libbmh:" in r.stderr
        assert not (tmp_path / "bib.decoded").exists()


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(BUILT), reason="integration/_build not built (needs /root/reference at build)")
def test_binding_compress_matches_reference_on_gpu(tmp_path):
    with open(os.path.join(GOLDEN, "calgary_stdout.json")) as f:
        tails = {e["file"]: e["stdout_tail"] for e in json.load(f)}
    for name, data, rec in golden_calgary():
        (tmp_path / name).write_bytes(data)
        r = subprocess.run([BUILT, name, name + ".bzap"], cwd=tmp_path, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert (tmp_path / (name + ".bzap")).read_bytes() == rec, name
        tree_len = int.from_bytes(rec[16:24], "little")
        assert r.stdout == f"header size: {24 + tree_len} $$ file_name: {name}.bzap $$ initial_data_size:" + tails[name]
    assert sorted(CALGARY) == sorted(tails)


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(BUILT), reason="integration/_build not built (needs /root/reference at build)")
def test_binding_decompress_decodes_on_gpu(tmp_path):
    """The binding's decompress() (main.cpp:327-345 against bmh_decompress_dev): every golden
    Calgary record (the reference's own bytes) decodes on the GPU back to the file."""
    dec = BUILT.replace("bmh_ref_compress", "bmh_ref_decompress")
    for name, data, rec in golden_calgary():
        (tmp_path / (name + ".bzap")).write_bytes(rec)
        r = subprocess.run([dec, name + ".bzap", name + ".decoded"], cwd=tmp_path, capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        assert (tmp_path / (name + ".decoded")).read_bytes() == data, name
