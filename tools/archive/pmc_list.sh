mkdir -p gpurun_out/pmc_list
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list/list.txt 2>&1
grep -o "SQ_[A-Z0-9_]*\|TA_[A-Z0-9_]*\|TCP_[A-Z0-9_]*\|TCC_[A-Z0-9_]*" gpurun_out/pmc_list/list.txt | sort -u > gpurun_out/pmc_list/names.txt
wc -l gpurun_out/pmc_list/names.txt
