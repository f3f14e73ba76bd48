import json, sys
for line in open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/ab.log'):
    line = line.strip()
    if line.startswith('{'):
        d = json.loads(line); r = d['runs'][-1]; r0 = d['runs'][1]
        print(d['N'], f"{r0['wall_s']*1e3:.1f}ms", f"{r0['mcells']:.0f}", 'passes', r['passes'], 'launch', r['launches'],
              'visits', r['tile_visits'], 'sweeps', r['inner_sweeps'], 'maxact', r['max_active'],
              'pass_ms', round(r['pass_ms'], 1), f"us/launch {r['pass_ms']*1e3/max(1,r['pass_launches']):.1f}", d['sumT'])
    elif 'passed' in line or line.startswith('v') or 'rc=' in line or 'Error' in line:
        print(line[:200])
