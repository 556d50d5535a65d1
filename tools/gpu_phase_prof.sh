set -o pipefail
mkdir -p gpurun_out/ph
for SC in lunar robocup; do
timeout -k 10 120 python tools/phase_prof.py --scenario $SC > gpurun_out/ph/$SC.json 2> gpurun_out/ph/$SC.err || { tail gpurun_out/ph/$SC.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ph/$SC.json'));print('$SC', round(d['cycles_per_wave_step_total']), {k:round(v['cycles_per_wave_step']) for k,v in d['phases'].items()})"
done
