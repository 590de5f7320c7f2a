import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            cpu = d.get('cpu_baseline', {}).get('value')
            print(f"{f}: value {d['value']:.4g} calls/s  step {d['roofline']['step']['ms']:.3f} ms ({d['roofline']['step']['GB/s']:.0f} GB/s)" + (f"  cpu {cpu:.0f}" if cpu else ""))
            for k, v in d['roofline']['kernels'].items():
                print(f"   {k:18s} {v['ms']:.4f} ms {v['GB/s']:7.0f} GB/s")
            if 'objective' in d:
                o = d['objective']
                print(f"   objective          {o['ms_per_batch']:.4f} ms {o['value']:.4g} calls/s")
            if 'gait_optimization' in d:
                o = d['gait_optimization']
                print(f"   gait_optimization  {o['ms_per_batch']:.4f} ms {o['value']:.4g} calls/s ({o['problems']} problems, nnz {o['nnz']}, {o['GB/s']:.0f} GB/s)")
