# A/B of the GRU loop's lookup layouts in the cfg2 forward: row layout (default below 1 GB
# volumes), sheared via the producers, and sheared + convc1 on MFMA; per-family live times.
set -e
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-epe"
timeout -k 10 300 $B > gpurun_out/abs_default.json
timeout -k 10 300 $B --opts shear_min_bytes=0,sheared_producers=1 > gpurun_out/abs_shp.json
timeout -k 10 300 $B --opts shear_min_bytes=0,sheared_producers=1 --lookup-mfma 1 > gpurun_out/abs_shpm.json
timeout -k 10 300 $B --lookup-mfma 1 > gpurun_out/abs_m.json
python3 - <<'PY'
import json
for n in ("default", "shp", "shpm", "m"):
    d = json.loads(open("gpurun_out/abs_%s.json" % n).read().strip().splitlines()[-1])
    k = d["roofline"]["kernels"]
    print(n, round(d["ms_per_step"], 2), round(d["roofline"]["one_stream_ms_per_step"], 2),
          {f: (round(k[f]["ms_per_step"], 3), round(k[f]["avg_launch_us"], 1)) for f in k
           if f in ("corr_lookup", "corr_shear", "corr_volume_pyramid", "mono_pyramid")})
PY
