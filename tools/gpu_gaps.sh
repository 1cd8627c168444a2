# Kernel-trace timeline of the timed PH steps (gaps between launches) + one bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_profile.sh > /dev/null || exit $?
python - <<'PY'
import csv
rows = sorted(csv.DictReader(open('gpurun_out/prof/trace/run_kernel_trace.csv')), key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'pdhg' in r['Kernel_Name']]
prev = None
for r in rows[idx[-5]:idx[-1] + 1]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"dur {(e - s) / 1e3:8.1f} gap {((s - prev) / 1e3 if prev else 0):6.1f}  {r['Kernel_Name'][:40]}")
    prev = e
PY
timeout -k 10 300 python -u bench.py --cpu-seconds 0 --conv-iters 0 > gpurun_out/bench_gap.json 2> gpurun_out/bench_gap.err
rc=$?; python -c "import json;d=json.load(open('gpurun_out/bench_gap.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"; exit $rc
