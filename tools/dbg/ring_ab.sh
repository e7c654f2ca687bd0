L="zlib-streams-ts_amd/libzsgpu.so variants/r256/libzsgpu.so variants/r512/libzsgpu.so"
bash tools/dbg/lib_ab.sh "--mode inflate --stream-bytes 262144 --replicas 1 --corpus text --streams 512" $L
bash tools/dbg/lib_ab.sh "--mode inflate --format gzip --replicas 1 --streams 8192" $L
bash tools/dbg/lib_ab.sh "--level 9 --streams 1024" zlib-streams-ts_amd/libzsgpu.so
bash tools/dbg/lib_ab.sh "--level 9 --streams 1024 --option match_sweep=0" zlib-streams-ts_amd/libzsgpu.so
