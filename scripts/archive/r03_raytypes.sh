HPT_TRACE_REPORT=1 timeout -k 10 300 python -u tools/ray_types_probe.py > gpurun_out/raytypes.log 2>&1; tail -20 gpurun_out/raytypes.log
