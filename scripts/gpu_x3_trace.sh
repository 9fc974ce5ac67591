export TMPDIR=/tmp; mkdir -p gpurun_out
export FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_tr.so
TRACE_CASES=c3_64_full,c3_128_half,c7_32_64_full,d3_128_half timeout -k 10 200 python scripts/x3_trace.py > gpurun_out/trace_base.txt 2>&1; cat gpurun_out/trace_base.txt
FVC_X3_WL=1 TRACE_CASES=c3_64_full,c3_128_half timeout -k 10 200 python scripts/x3_trace.py > gpurun_out/trace_wl.txt 2>&1; cat gpurun_out/trace_wl.txt
