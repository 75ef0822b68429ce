#!/usr/bin/env python3
"""One line per bench.py JSON under DIR and DIR/emu (ms per step, per frame of work, launch shape, heavy
pixels, per-rank trace / exchange device time).  Usage: emu_table.py DIR"""
import json,glob,os,sys
def load(f):
    l=[x for x in open(f) if x.startswith('{')]
    return json.loads(l[-1]) if l else None
d0=sys.argv[1]
for f in sorted(glob.glob(d0+'/*.json'))+sorted(glob.glob(d0+'/emu/*.json')):
    d=load(f)
    if not d: print(f,'FAIL'); continue
    r=d['roofline']; c=d['config']
    p=d['per_rank'][0]
    n=int(f.split('_n')[-1].split('_')[0]) if '_n' in os.path.basename(f) and '/emu/' in f else 1
    per_work = d['ms_per_step']*n/c['frames_per_step']
    print(f"{os.path.basename(f):26s} ms/step {d['ms_per_step']:.4f} per-frame-work {per_work:.4f} F{c['frames_per_launch']} D{c['launches_in_flight']} G{c['exchange_every_frames']} kms {r['kernel_ms']:.3f} fdev {r['frame_ms_device']:.4f} infl {r['launches_in_flight_avg']} hpx {c['schedule']['heavy_pixels_used']} busy {p['trace_busy_ms_per_frame']} exch {p['exchange_ms_per_frame']}")
