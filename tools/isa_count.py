"""Static instruction counts of the product kernels (device ISA of dct3d_kernels.hip, built here).

    python tools/isa_count.py [kernel-substring ...]

Prints, per kernel: VALU / fp64 VALU / SALU / LDS / VMEM instruction counts of the whole function
(every path, rare ones included), the VGPR count and the scratch size.  A quick A/B of a kernel
change's issue cost before spending a GPU run on it."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "3ddctvideoencoding_amd", "csrc", "dct3d_kernels.hip")


def main():
    out = "/tmp/dct3d_isa.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                           "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S", "-o", out, SRC],
                          stderr=subprocess.DEVNULL)
    s = open(out).read()
    want = sys.argv[1:] or ["decode_kernel", "decode_eg_kernel", "encode16_kernel"]
    for m in re.finditer(r"^(_Z\S+):\s", s, re.M):
        name = m.group(1)
        if not any(w in name for w in want):
            continue
        end = s.index(".Lfunc_end", m.end())
        body = s[m.end():end]
        ops = collections.Counter(re.findall(r"^\s+([vsdgbf]\w+|scratch_\w+)", body, re.M))
        valu = sum(v for k, v in ops.items() if k.startswith("v_"))
        f64 = sum(v for k, v in ops.items() if k.startswith("v_") and "f64" in k)
        salu = sum(v for k, v in ops.items() if k.startswith("s_"))
        lds = sum(v for k, v in ops.items() if k.startswith("ds_"))
        vmem = sum(v for k, v in ops.items() if k.startswith(("global_", "buffer_", "scratch_", "flat_")))
        k0 = s.find(".amdhsa_kernel " + name + "\n")
        meta = s[k0:s.index(".end_amdhsa_kernel", k0)] if k0 >= 0 else ""
        vg = re.search(r"amdhsa_next_free_vgpr (\d+)", meta)
        pr = re.search(r"amdhsa_private_segment_fixed_size (\d+)", meta)
        print(f"{name[:70]:70s} valu {valu:5d} f64 {f64:4d} salu {salu:4d} lds {lds:3d} vmem {vmem:3d} "
              f"vgpr {vg.group(1) if vg else '-'} scratch {pr.group(1) if pr else '-'}")


if __name__ == "__main__":
    main()
