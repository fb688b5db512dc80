set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for t in r03 t_9d22582 t_a645a35 t_56894d1 t_258fdcb head; do
    if [ $t = head ]; then d=.; else d=tools/ab/$t; fi
    (cd $d && timeout -k 10 300 python -u tools/rewalk_probe.py --batches 6) > gpurun_out/bi_${t}_$rep.log 2>&1
    echo "$t rep $rep: $(tail -1 gpurun_out/bi_${t}_$rep.log | cut -c1-120)"
  done
done
