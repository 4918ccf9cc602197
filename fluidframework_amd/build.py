"""Build libmtgpu.so (gfx950) in-tree with hipcc.  No GPU needed to build."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
LIB = os.path.join(HERE, 'libmtgpu.so')
SOURCES = ['mt_apply.hip', 'mt_apply_reg.hip', 'mt_service.hip', 'mt_deli.hip', 'mt_engine.cpp', 'mt_comm.cpp']
HEADERS = ['mt_state.h', 'mt_wave.h', 'mt_checksum.h', 'mt_synth.h', '../../include/mtgpu.h']
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('PYTORCH_ROCM_ARCH', 'gfx950')


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in SOURCES + HEADERS
               if os.path.exists(os.path.join(CSRC, f)))


def build(force=False, verbose=False, prof=False):
    """Compile every source to an object in parallel (hipcc, gfx950), then link libmtgpu.so.
    prof=True builds the diagnostic libmtgpu_prof.so (-DMT_PROF per-phase cycle stamps)."""
    lib = LIB.replace('libmtgpu.so', 'libmtgpu_prof.so') if prof else LIB
    if not prof and not force and not needs_build():
        return LIB
    from concurrent.futures import ThreadPoolExecutor
    objdir = os.path.join(HERE, 'build')
    os.makedirs(objdir, exist_ok=True)
    srcs = [f for f in SOURCES if os.path.exists(os.path.join(CSRC, f))]
    flags = [f'--offload-arch={ARCH}', '-O3', '-std=c++17', '-fPIC', '-Wall', '-Wno-unused-function',
             '-Wno-unused-result', '-Wno-unused-value'] + os.environ.get('MTGPU_EXTRA_FLAGS', '').split()

    stamp = ' '.join(flags + (['-DMT_PROF'] if prof else []))
    hdr_t = max(os.path.getmtime(os.path.join(CSRC, h)) for h in HEADERS if os.path.exists(os.path.join(CSRC, h)))

    def fresh(f, obj):
        # an object is reused when it is newer than its source and every header, and was built
        # with the same flags (recorded next to it)
        try:
            t = os.path.getmtime(obj)
            with open(obj + '.flags') as fh:
                same = fh.read() == stamp
        except OSError:
            return False
        return same and t > os.path.getmtime(os.path.join(CSRC, f)) and t > hdr_t

    def cc(f):
        obj = os.path.join(objdir, f + ('.prof.o' if prof else '.o'))
        if not force and fresh(f, obj):
            return obj
        cmd = [HIPCC] + flags + (['-DMT_PROF'] if prof else []) + ['-c', os.path.join(CSRC, f), '-o', obj]
        if verbose:
            print(' '.join(cmd))
        subprocess.check_call(cmd)
        with open(obj + '.flags', 'w') as fh:
            fh.write(stamp)
        return obj

    with ThreadPoolExecutor(max_workers=len(srcs)) as ex:
        objs = list(ex.map(cc, srcs))
    # RCCL (the end-of-run checksum gather, mt_comm.cpp) from /opt/rocm
    subprocess.check_call([HIPCC, f'--offload-arch={ARCH}', '-shared', '-o', lib + '.tmp'] + objs +
                          ['-L/opt/rocm/lib', '-lrccl', '-Wl,-rpath,/opt/rocm/lib'])
    os.replace(lib + '.tmp', lib)
    return lib


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
    if '--prof' in sys.argv:
        print(build(prof=True, verbose=True))
        sys.exit(0)
    build(force='-f' in sys.argv, verbose=True)
    build_napi(force=True)
    print(LIB)
