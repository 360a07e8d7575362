"""Static VALU budget of ransac_fit_kernel<float> by phase, from the gfx950 ISA of ablation builds
(VERDICT r3 item 5).  Each phase's count = full build minus the build with that phase removed
(RANSAC_ABL_* knobs in csrc/ransac.hip; timing-only builds, results invalid).  The preview loop
runs PV / 8 iterations of an 8-match body, so its dynamic count is scaled from the static one.

Usage: python tools/isa_fit_budget.py  -> one JSON line (counts per wave = per 64 hypotheses).
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "sfm-project_amd", "csrc", "ransac.hip")
FL = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-gpu-rdc",
      "-fno-slp-vectorize", "--cuda-device-only", "-S"]
KERNEL = "ransac_fit_kernelIfE"
FMA = ("v_fma_f32", "v_fmac_f32", "v_mul_f32", "v_pk_fma_f32", "v_pk_mul_f32", "v_add_f32",
       "v_sub_f32")


def counts(defs):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "r.s")
        subprocess.run(["/opt/rocm/bin/hipcc"] + FL + [f"-D{d}" for d in defs] + [SRC, "-o", out],
                       check=True, stderr=subprocess.DEVNULL)
        s = open(out).read()
    name = re.search(r"^(_Z\w*" + KERNEL + r"\w*):", s, re.M).group(1)
    body = s[s.index(name + ":"):]
    body = body[:body.index(".Lfunc_end")]
    ops = [l.split()[0] for l in (x.strip() for x in body.splitlines())
           if l and not l.startswith((".", ";")) and not l.endswith(":")]
    c = collections.Counter(ops)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    fma = sum(v for k, v in c.items() if k.startswith(FMA))
    # the preview's loop body: instructions between the loop label and its back-branch
    return {"valu": valu, "fma_family": fma, "salu": sum(v for k, v in c.items() if k.startswith("s_")),
            "vmem": sum(v for k, v in c.items() if k.startswith(("global_", "buffer_"))),
            "div_seq": c.get("v_div_fixup_f32", 0), "sqrt": c.get("v_sqrt_f32_e32", 0),
            "mad_u64": c.get("v_mad_u64_u32", 0), "ldexp": c.get("v_ldexp_f32", 0)}


def main():
    full = counts([])
    abl = {k: counts([d]) for k, d in (("sample", "RANSAC_ABL_NOSAMPLE"),
                                       ("fit", "RANSAC_ABL_NOFIT"),
                                       ("rank2", "RANSAC_ABL_NORANK2"),
                                       ("preview", "RANSAC_ABL_NOPREVIEW"))}
    phases = {k: {m: full[m] - v[m] for m in ("valu", "fma_family")} for k, v in abl.items()}
    phases["rest (scales, gathers, record store, address math)"] = {
        m: full[m] - sum(phases[k][m] for k in ("sample", "fit", "preview")) for m in ("valu", "fma_family")}
    print(json.dumps({"kernel": "ransac_fit_kernel<float>", "static_full": full,
                      "static_by_phase": phases,
                      "note": "fit = QR + back-substitution + rank 2; rank2 is the part of fit after "
                              "the null vector; static counts (the preview is a loop of PV/8 "
                              "8-match iterations: dynamic = static + (PV/8 - 1) x body)"}))


if __name__ == "__main__":
    main()
