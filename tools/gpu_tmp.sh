bash tools/gpu_libab.sh tex lib lib_park && SKIP_TESTS=1 bash tools/gpu_libab.sh tex2 lib lib_prev lib_park && SKIP_TESTS=1 bash tools/gpu_ab.sh tex7 "PT_MIN_WAVES=7" "PT_MIN_WAVES=6"
