"""Builds the plain-C hosts of include/hgd.h under examples/ with gcc."""
import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hypergraph_diffusion_for_recommendation_amd", "_lib")


def build(out_path, source="hgconv2_host.c"):
    gcc = shutil.which("gcc")
    if gcc is None:
        return None
    cmd = [gcc, "-std=c11", "-Wall", "-Werror", "-O2", "-D__HIP_PLATFORM_AMD__",
           "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
           os.path.join(ROOT, "examples", source), "-L", LIB, "-lhgd",
           "-L", "/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{LIB}", "-Wl,-rpath,/opt/rocm/lib",
           "-lm", "-o", str(out_path)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return str(out_path)
