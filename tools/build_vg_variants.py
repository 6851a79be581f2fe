"""Build _hip_ops variants that differ only in how value_grad.hip is compiled (LLVM scheduler
options), each as a self-contained package copy under build_variants/<name>/ with its own
tools/kbench.py, so `python build_variants/<name>/tools/kbench.py grad` times that build.
Run after the normal build (reuses build/hip/*.o for every other object)."""
import glob
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from relayrl_prototype_amd import _build as B  # noqa: E402

VARIANTS = {
    "base": [],
    "maxilp": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    "trackers": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
    "bias0": ["-mllvm", "-amdgpu-schedule-metric-bias=0"],
}


def main():
    kdir = os.path.join(B.CSRC, "kernels")
    src = os.path.join(kdir, "value_grad.hip")
    others = [o for o in glob.glob(os.path.join(B.BUILD, "hip", "*.o")) if not o.endswith("value_grad.hip.o")]
    tinc, tcf, tld = B._torch_flags()
    so_name = os.path.basename(B.HIP_OPS)
    for name, extra in VARIANTS.items():
        root = os.path.join(REPO, "build_variants", name)
        pkg = os.path.join(root, "relayrl_prototype_amd")
        if os.path.exists(root):
            shutil.rmtree(root)
        shutil.copytree(os.path.join(REPO, "relayrl_prototype_amd"), pkg,
                        ignore=shutil.ignore_patterns("__pycache__", "_hip_ops*.so"))
        os.makedirs(os.path.join(root, "tools"))
        shutil.copy(os.path.join(REPO, "tools", "kbench.py"), os.path.join(root, "tools", "kbench.py"))
        obj = os.path.join(root, "value_grad.hip.o")
        cmd = [B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
               *B.HIP_FLAGS, *extra, "-I", kdir, "-c", src, "-o", obj]
        subprocess.run(cmd, check=True)
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-pthread", obj] + others +
                       ["-o", os.path.join(pkg, so_name)] + tld, check=True)
        os.remove(obj)
        print("built", name, flush=True)


if __name__ == "__main__":
    main()
