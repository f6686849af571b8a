"""Summarise one training step from a rocprofv3 kernel trace: the last N
dispatches of the k-th occurrence of the step's marker kernel.  Prints
per-dispatch duration, grid and VGPRs for kernels matching a pattern.
usage: trace_step.py <dir> <pattern> [step_index_from_end]"""
import csv
import re
import sys

d, pat = sys.argv[1], sys.argv[2]
back = int(sys.argv[3]) if len(sys.argv) > 3 else 2
rows = list(csv.DictReader(open(d + '/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# step boundary: the Adam kernel ends each step
ends = [i for i, r in enumerate(rows) if 'adam_kernel' in r['Kernel_Name']]
s0, s1 = ends[-back - 1] + 1, ends[-back] + 1
step = rows[s0:s1]
tot = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in step)
span = int(step[-1]['End_Timestamp']) - int(step[0]['Start_Timestamp'])
print(f'step dispatches {len(step)}  kernel time {tot/1e6:.3f} ms  span {span/1e6:.3f} ms')
rx = re.compile(pat)
agg = {}
for r in step:
    name = r['Kernel_Name']
    if not rx.search(name):
        continue
    dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    short = re.sub(r'\(anonymous namespace\)::', '', name)[:70]
    g = (int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']), int(r['Grid_Size_Y']), int(r['Grid_Size_Z']))
    print(f'{dur:9.1f} us  grid {g}  vgpr {r["VGPR_Count"]}/{r["Accum_VGPR_Count"]}  lds {r["LDS_Block_Size"]}  {short}')
