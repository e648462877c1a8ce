"""VGPRs and scratch of every kernel in a .hip file (hipcc --save-temps), e.g. before / after a change:
    python tools/kstats.py fl_sim_amd/csrc/topk.hip [filter]
    git show HEAD:fl_sim_amd/csrc/topk.hip > /tmp/old.hip && python tools/kstats.py /tmp/old.hip"""
import glob
import os
import re
import subprocess
import sys
import tempfile

src = os.path.abspath(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
inc = [f"-I{os.path.dirname(os.path.abspath(__file__))}/../include",
       f"-I{os.path.dirname(os.path.abspath(__file__))}/../fl_sim_amd/csrc"]
with tempfile.TemporaryDirectory() as d:
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", *inc,
                    "--save-temps", "-c", src, "-o", f"{d}/k.o"],
                   cwd=d, check=True, stderr=subprocess.DEVNULL)
    s = open(glob.glob(f"{d}/*gfx950*.s")[0]).read()
for b in s.split(".end_amdhsa_kernel"):
    nm = re.search(r"\.amdhsa_kernel (\S+)", b)
    if not nm or flt not in nm.group(1):
        continue
    ps = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", b).group(1)
    vg = re.search(r"\.amdhsa_next_free_vgpr (\d+)", b).group(1)
    print(f"scratch {ps:>4}  vgpr {vg:>4}  {nm.group(1)[:120]}")
