"""Build libmtgpu.so (gfx950) in-tree with hipcc.  No GPU needed to build."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
LIB = os.path.join(HERE, 'libmtgpu.so')
SOURCES = ['mt_apply.hip', 'mt_service.hip', 'mt_synth.hip', 'mt_engine.cpp']
HEADERS = ['mt_state.h', 'mt_wave.h', 'mt_checksum.h', 'mt_synth.h', '../../include/mtgpu.h']
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('PYTORCH_ROCM_ARCH', 'gfx950')


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in SOURCES + HEADERS
               if os.path.exists(os.path.join(CSRC, f)))


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB
    srcs = [os.path.join(CSRC, f) for f in SOURCES if os.path.exists(os.path.join(CSRC, f))]
    cmd = [HIPCC, f'--offload-arch={ARCH}', '-O3', '-std=c++17', '-fPIC', '-shared', '-Wall',
           '-Wno-unused-function', '-o', LIB + '.tmp'] + srcs
    if verbose:
        print(' '.join(cmd))
    subprocess.check_call(cmd)
    os.replace(LIB + '.tmp', LIB)
    return LIB


JS = os.path.join(os.path.dirname(HERE), 'js')
NAPI = os.path.join(JS, 'mtgpu.node')


def build_napi(force=False):
    """The Node N-API addon (js/mtgpu.node) over libmtgpu.so, if node's headers are present."""
    inc = '/usr/include/node'
    src = os.path.join(JS, 'mtgpu_napi.c')
    if not os.path.exists(os.path.join(inc, 'node_api.h')):
        return None
    if not force and os.path.exists(NAPI) and os.path.getmtime(NAPI) >= max(os.path.getmtime(src),
                                                                            os.path.getmtime(LIB)):
        return NAPI
    subprocess.check_call(['gcc', '-O2', '-fPIC', '-shared', '-Wall', '-Wno-unused-parameter',
                           '-DNODE_GYP_MODULE_NAME=mtgpu', f'-I{inc}', '-o', NAPI, src, f'-L{HERE}',
                           '-l:libmtgpu.so', "-Wl,-rpath,$ORIGIN/../fluidframework_amd"])
    return NAPI


if __name__ == '__main__':
    build(force='-f' in sys.argv, verbose=True)
    build_napi(force=True)
    print(LIB)
