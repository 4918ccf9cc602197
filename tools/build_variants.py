#!/usr/bin/env python3
"""Build A/B variants of libmtgpu.so (diagnostic tooling): each variant recompiles the register
engine (mt_apply_reg.hip) with its own -D flags and links it with the in-tree objects of the other
sources (fluidframework_amd/build/*.o, from a normal build).  Output: ablib/libmtgpu_<name>.so, for
tools/ab.py on the GPU box.
    python tools/build_variants.py base= new=-DMT_FOO 'both=-DMT_FOO -DMT_BAR'"""
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'fluidframework_amd')
HIPCC = '/opt/rocm/bin/hipcc'
FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-Wall', '-Wno-unused-function', '-Wno-unused-result',
         '-Wno-unused-value']


# the sources are snapshotted first: hipcc reads the file once per compilation pass (device, then
# host), so an edit made while a variant builds would otherwise split one object between two versions
SNAP = tempfile.mkdtemp(prefix='mtgpu_variants_')
shutil.copytree(os.path.join(PKG, 'csrc'), os.path.join(SNAP, 'fluidframework_amd', 'csrc'))
shutil.copytree(os.path.join(REPO, 'include'), os.path.join(SNAP, 'include'))


def build_one(spec):
    name, _, defs = spec.partition('=')
    out = os.path.join(REPO, 'ablib')
    os.makedirs(out, exist_ok=True)
    obj = os.path.join(out, f'mt_apply_reg_{name}.o')
    src = os.path.join(SNAP, 'fluidframework_amd', 'csrc', 'mt_apply_reg.hip')
    subprocess.check_call([HIPCC] + FLAGS + defs.split() + ['-c', src, '-o', obj])
    others = [os.path.join(PKG, 'build', f + '.o') for f in
              ('mt_apply.hip', 'mt_service.hip', 'mt_deli.hip', 'mt_engine.cpp', 'mt_comm.cpp')]
    lib = os.path.join(out, f'libmtgpu_{name}.so')
    subprocess.check_call([HIPCC, '--offload-arch=gfx950', '-shared', '-o', lib, obj] + others +
                          ['-L/opt/rocm/lib', '-lrccl', '-Wl,-rpath,/opt/rocm/lib'])
    return lib


if __name__ == '__main__':
    with ThreadPoolExecutor(max_workers=4) as ex:
        for lib in ex.map(build_one, sys.argv[1:]):
            print(lib)
