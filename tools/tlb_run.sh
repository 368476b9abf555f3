export TMPDIR=/tmp
O=gpurun_out/tlb
mkdir -p $O
timeout -k 10 120 ./tools/alloc_ab 10 sweep 12 > $O/plain.jsonl 2> $O/plain.err &&
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum --output-format csv -d $O/pmc_tlb -o run -- ./tools/alloc_ab 2 sweep 12 > $O/alloc_tlb.jsonl 2> $O/alloc_tlb.err &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $O/pmc_ea -o run -- ./tools/alloc_ab 2 sweep 12 > $O/alloc_ea.jsonl 2> $O/alloc_ea.err
echo done
