"""Build libigr.so (HIP, gfx950) in-tree: inductive-recommendation_amd/igr/lib/libigr.so.

Each source is compiled with hipcc into build/<name>.o (skipped when newer
than its inputs) and linked into one shared library exporting the C ABI of
include/igr.h.  No JIT cache: the .so travels with the repository snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
INCLUDE = os.path.join(ROOT, 'include')
OBJ = os.path.join(HERE, 'build')
LIB = os.path.join(HERE, 'igr', 'lib', 'libigr.so')
SOURCES = ['spmm.hip', 'spmm_rows.hip', 'topk.hip', 'edge_ops.hip', 'att_shared.hip', 'bpr.hip', 'rowsort.hip', 'gemm.hip', 'linear_wgrad.hip', 'train_ops.hip', 'graph_host.cpp', 'capi.cpp']
ARCH = os.environ.get('IGR_OFFLOAD_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
# Packed fp32 VALU ops are switched off for the device pass (some of their
# forms have given wrong results on this hardware); the host pass warns that
# it does not know the feature, which is harmless.
CFLAGS = ['-O3', '-std=c++17', '-fPIC', f'--offload-arch={ARCH}', '-I', INCLUDE, '-I', CSRC,
          '-Xclang', '-target-feature', '-Xclang', '-packed-fp32-ops',
          '-Wall', '-Wno-unused-function'] + os.environ.get('IGR_EXTRA_CFLAGS', '').split()


def _newer(target, deps):
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def build(verbose=False, jobs=8, lib=None, obj=None):
    """Compile and link; `lib`/`obj` override the output paths (tuning variants)."""
    global LIB, OBJ
    LIB, OBJ = lib or LIB, obj or OBJ
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    headers = [os.path.join(CSRC, 'common.h'), os.path.join(CSRC, 'segsum.h'), os.path.join(INCLUDE, 'igr.h')]
    objs, procs = [], []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, os.path.splitext(src)[0] + '.o')
        objs.append(o)
        if _newer(o, [s] + headers):
            continue
        cmd = [HIPCC] + CFLAGS + ['-x', 'hip', '-c', s, '-o', o]
        if verbose:
            print(' '.join(cmd), flush=True)
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        if len(procs) >= jobs:
            _wait(procs.pop(0))
    for p in procs:
        _wait(p)
    if not _newer(LIB, objs):
        cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-o', LIB] + objs + ['-lpthread']
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.check_call(cmd)
    return LIB


def _wait(item):
    src, p = item
    out, _ = p.communicate()
    if p.returncode != 0:
        sys.stderr.write(out.decode(errors='replace'))
        raise RuntimeError(f'hipcc failed on {src}')
    # the host pass does not know the device-only target feature of CFLAGS
    txt = '\n'.join(ln for ln in out.decode(errors='replace').splitlines()
                    if "'-packed-fp32-ops' is not a recognized feature" not in ln).strip()
    if txt:
        sys.stderr.write(txt + '\n')


if __name__ == '__main__':
    print(build(verbose=True))
