"""Build the in-tree HIP library t2omca_amd/lib/libt2omca.so for gfx950.

    python -m t2omca_amd.build        (or __graft_entry__.build())

Every csrc/*.hip translation unit is compiled to an object in parallel and
linked into a single C-ABI shared library (declared in include/t2omca.h).  The .so is git-ignored
but travels to the GPU box inside the repo snapshot.
"""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libt2omca.so")
ARCH = os.environ.get("T2O_OFFLOAD_ARCH", "gfx950")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.hpp"))
    deps.append(os.path.join(os.path.dirname(HERE), "include", "t2omca.h"))
    return any(os.path.getmtime(p) > t for p in deps)


def build(force=False, verbose=False, jobs=None, out=None):
    """Compile each translation unit to an object in parallel, then link the .so
    (to `out` instead of the package library when given)."""
    if out is None and not force and not _stale():
        return LIB
    target = out or LIB
    os.makedirs(LIBDIR, exist_ok=True)
    objdir = os.path.join(LIBDIR, "obj" if out is None else "obj_" + os.path.basename(out))
    os.makedirs(objdir, exist_ok=True)
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++20", "-fPIC", "-Wno-unused-result"]
    objs, procs = [], []
    headers = glob.glob(os.path.join(CSRC, "*.hpp")) + [os.path.join(os.path.dirname(HERE), "include", "t2omca.h")]
    newest_header = max(os.path.getmtime(h) for h in headers)
    for src in sources():
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        # an object newer than its source, every header and this file is reused
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > max(
                os.path.getmtime(src), newest_header, os.path.getmtime(__file__)):
            continue
        cmd = [hipcc] + flags + ["-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd))
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    failed = False
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed = True
            sys.stderr.write(out)
        elif verbose and out.strip():
            sys.stderr.write(out)
    if failed:
        raise RuntimeError("hipcc failed building libt2omca.so")
    tmp = target + ".tmp"
    r = subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs,
                       capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("hipcc failed linking libt2omca.so")
    os.replace(tmp, target)
    return target


if __name__ == "__main__":
    out = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--out=")), None)
    print(build(force="--force" in sys.argv, verbose=True, out=out))
