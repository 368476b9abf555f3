# lone-burst stage breakdown (GCL_LOOP_STAMPS) + the shallow pipeline rows
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/${1:-r04c}_stages.jsonl
for a in "64 records" "1 records" "64 offsets" "1 offsets"; do
  set -- $a
  RXPIPE_STAMPS=1 timeout -k 10 60 tools/rxpipe $1 1 1 20000 $( [ $2 = records ] && echo records ) >> $out || exit 1
done
for a in "64 4 8 20000" "64 4 8 20000 records" "64 8 16 40000 records" "64 16 32 40000"; do
  timeout -k 10 60 tools/rxpipe $a >> $out || exit 1
done
cat $out
