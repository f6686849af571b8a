#!/usr/bin/env python3
"""Compile one csrc file for gfx950 and print per-kernel VGPR/AGPR, scratch,
LDS and occupancy from -Rpass-analysis=kernel-resource-usage.
usage: python tools/kres.py halo_conv.hip [name-filter]"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, 'uncertainty-model_amd', 'csrc')


def main():
    src = os.path.join(CSRC, sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ''
    cmd = ['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '--offload-arch=gfx950',
           '-I', os.path.join(REPO, 'include'), '-I', CSRC, '-c', src, '-o', '/tmp/kres.o',
           '-Rpass-analysis=kernel-resource-usage']
    r = subprocess.run(cmd, capture_output=True, text=True)
    cur = None
    rows = []
    for line in r.stderr.splitlines():
        m = re.search(r'remark: (.*?) \[-Rpass', line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith('Function Name:'):
            cur = {'name': t.split(':', 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ':' in t:
            k, v = t.split(':', 1)
            cur[k.strip()] = v.strip()
    for d in rows:
        if filt and filt not in d['name']:
            continue
        n = re.sub(r'_ZN12_GLOBAL__N_1\d+', '', d['name'])[:70]
        print(f"{n:70s} vgpr {d.get('VGPRs', '?'):>4} agpr {d.get('AGPRs', '?'):>4} "
              f"scratch {d.get('ScratchSize [bytes/lane]', '?'):>4} "
              f"lds {d.get('LDS Size [bytes/block]', '?'):>6} occ {d.get('Occupancy [waves/SIMD]', '?')}")
    if r.returncode:
        print(r.stderr[-3000:])


if __name__ == '__main__':
    main()
