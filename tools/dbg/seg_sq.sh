set -u
timeout -k 10 600 tools/pmc_sq.sh gpurun_out/sq_c5i --mode inflate --format gzip --streams 8192 --replicas 1 && \
python3 tools/sq_summary.py gpurun_out/sq_c5i zs_k_seg && \
timeout -k 10 600 tools/pmc_sq.sh gpurun_out/sq_c4d512 --mode inflate --stream-bytes 262144 --streams 512 --replicas 1 --corpus text && \
python3 tools/sq_summary.py gpurun_out/sq_c4d512 zs_k_seg
