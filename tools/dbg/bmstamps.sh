export ME_MFMA_BM=1; timeout -k 10 120 python3 tools/mfma_stamps.py 1080p > gpurun_out/st1080.txt 2>&1; head -5 gpurun_out/st1080.txt; timeout -k 10 120 python3 tools/mfma_stamps.py 4k 2>&1 | head -8
