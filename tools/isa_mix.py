"""Static instruction mix of the gfx950 kernels in one compiled object (csrc/*.o).

  python tools/isa_mix.py deep-learning-...-attention_amd/csrc/fused.o --match ru_stream

Extracts the object's HIP fat binary, unbundles the gfx950 code object, disassembles it
(llvm-objdump) and counts, per kernel, MFMAs, VALU (packed / transcendental split out), LDS,
global and scalar instructions, plus an issue-cost estimate of one wave's vector stream from the
MI355X_MICROARCH issue-cost table (4 cycles per VALU / packed-f32 op, 8 per transcendental,
8 per 16x16x32 MFMA).  The hot kernels here are fully unrolled, so the static counts are the
per-wave dynamic counts.
"""
import argparse
import os
import re
import subprocess
import tempfile
from collections import Counter

LLVM = "/opt/rocm/lib/llvm/bin"
TRANS = {"v_exp_f32_e32", "v_rcp_f32_e32", "v_log_f32_e32", "v_rsq_f32_e32", "v_sqrt_f32_e32",
         "v_exp_f32_e64", "v_rcp_f32_e64", "v_log_f32_e64", "v_rsq_f32_e64", "v_sqrt_f32_e64"}


def disassemble(obj):
    d = tempfile.mkdtemp()
    fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj,
                    os.path.join(d, "x.o")], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "-C", co], check=True,
                          capture_output=True, text=True).stdout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("obj")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    for f in re.split(r"\n(?=[0-9a-f]{16} <)", disassemble(a.obj)):
        m = re.match(r"[0-9a-f]+ <(.+)>:", f)
        if not m or a.match not in m.group(1):
            continue
        ins = [ln.strip().split()[0] for ln in f.split("\n")[1:]
               if ln.strip() and not ln.strip().startswith((";", "//"))]
        c = Counter(ins)
        n = lambda p: sum(v for k, v in c.items() if p(k))
        mfma = n(lambda k: k.startswith("v_mfma"))
        trans = n(lambda k: k in TRANS)
        pk = n(lambda k: k.startswith("v_pk_"))
        valu = n(lambda k: k.startswith("v_") and not k.startswith("v_mfma"))
        issue = 4 * (valu - trans) + 8 * trans + 8 * mfma
        print(f"{m.group(1)[:90]}\n  instructions {len(ins)}  mfma {mfma}  valu {valu} "
              f"(packed {pk}, transcendental {trans})  ds {n(lambda k: k.startswith('ds_'))}  "
              f"global {n(lambda k: k.startswith('global_') or k.startswith('buffer_'))}  "
              f"scalar {n(lambda k: k.startswith('s_'))}\n"
              f"  vector issue estimate {issue} cycles/wave (MFMA pipe {16 * mfma} cycles/wave "
              f"for 16x16x32)")


if __name__ == "__main__":
    main()
