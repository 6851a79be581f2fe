# value_grad.hip scheduler-option variants (tools/build_vg_variants.py): value and policy step
# kernels at the flagship shape, variants alternated twice.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/vg_variants.jsonl
for r in 1 2; do
  for v in base maxilp trackers bias0; do
    timeout -k 10 120 python build_variants/$v/tools/kbench.py grad --B 2097152 --iters 20 > gpurun_out/vg_$v.json 2>&1 || exit $?
    timeout -k 10 120 python build_variants/$v/tools/kbench.py pgrad --B 2097152 --iters 10 > gpurun_out/vgp_$v.json 2>&1 || exit $?
    echo "{\"variant\": \"$v\", \"round\": $r, \"grad\": $(grep -h '^{' gpurun_out/vg_$v.json | tail -1), \"pgrad\": $(grep -h '^{' gpurun_out/vgp_$v.json | tail -1)}" | tee -a gpurun_out/vg_variants.jsonl | cut -c1-260
  done
done
