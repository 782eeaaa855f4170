"""CPU: the register and LDS budgets the headline kernels' occupancy depends on,
read from the gfx950 code objects hipcc produces for csrc/*.hip. A kernel that crosses a budget
loses a workgroup per CU (round 5: k_finish_dense at 65 VGPRs ran 3.3 -> 3.6 ms per GiB)."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "bwt-mtf-huffman-compressor_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

# kernel (mangled-name fragment) -> (max VGPRs, max LDS bytes): 512-thread k_finish_dense needs
# <= 64 VGPRs and <= 40 KB for 4 workgroups per CU; 1024-thread k_g1_scatter <= 64 VGPRs and
# <= 80 KB for 2; one-wave k_mtf_encode <= 23.6 KB for 6 (and <= 256 VGPRs: 2 waves per SIMD)
BUDGETS = {
    "bwt.hip": {"k_finish_denseILj512ELj4608": (64, 40960), "k_g1_scatter": (64, 81920)},
    "mtf.hip": {"k_mtf_encode": (256, 24 * 1024)},
}


def _kernels(src: str) -> dict:
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run([HIPCC, "-O3", "-std=c++17", "-I", os.path.join(REPO, "include"), "-I", CSRC,
                        "--offload-arch=gfx950", "--cuda-device-only", "-S", "-o", out, os.path.join(CSRC, src)],
                       check=True, capture_output=True)
        s = open(out).read()
    res = {}
    for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", s, re.S):
        res[m.group(1)] = (int(re.search(r"next_free_vgpr (\d+)", m.group(2)).group(1)),
                           int(re.search(r"group_segment_fixed_size (\d+)", m.group(2)).group(1)))
    return res


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc absent")
@pytest.mark.parametrize("src", sorted(BUDGETS))
def test_kernel_register_and_lds_budgets(src):
    ks = _kernels(src)
    for frag, (vmax, lmax) in BUDGETS[src].items():
        hits = [(n, v) for n, v in ks.items() if frag in n]
        assert hits, frag
        for n, (v, lds) in hits:
            assert v <= vmax, (n, v, vmax)
            assert lds <= lmax, (n, lds, lmax)
