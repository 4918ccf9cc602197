#!/usr/bin/env python3
"""Per-kernel resource usage of the register apply engine as the compiler reports it
(-Rpass-analysis=kernel-resource-usage, gfx950): VGPRs, SGPRs, scratch bytes per lane (spills),
occupancy.  rocprofv3's kernel-trace "VGPR" column is half the compiler's arch VGPR count rounded
to its granule (e.g. K = 9: 226 here, 116 in profiles/r02_kernel_stats_C3_v2.csv).
    python tools/resource_usage.py > profiles/r02_resource_usage_reg.txt"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, 'fluidframework_amd', 'csrc', 'mt_apply_reg.hip')


def main():
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-Wno-unused-value',
                            '--cuda-device-only', '-Rpass-analysis=kernel-resource-usage', '-c', SRC, '-o',
                            os.path.join(d, 'o')], capture_output=True, text=True, check=True)
    print('# mt_apply_reg.hip, hipcc -O3 --offload-arch=gfx950 -Rpass-analysis=kernel-resource-usage')
    print('# %-8s %6s %6s %14s %10s' % ('kernel', 'VGPR', 'SGPR', 'scratch B/lane', 'waves/SIMD'))
    for b in re.split(r'remark: [^\n]*Function Name: ', r.stderr)[1:]:
        m = re.search(r'reg_apply_kernel(_c64|_ev)?ILi(\d+)E', b.split('\n')[0])
        if not m:
            continue
        kname = {'_c64': 'c64 K=', '_ev': 'ev K='}.get(m.group(1), 'K=') + m.group(2)

        def g(k):
            x = re.search(k + r': (\S+)', b)
            return x.group(1) if x else '?'
        print('  %-8s %6s %6s %14s %10s' % (kname, g('VGPRs'), g('SGPRs'), g(r'ScratchSize \[bytes/lane\]'),
                                            g(r'Occupancy \[waves/SIMD\]')))


if __name__ == '__main__':
    sys.exit(main())
