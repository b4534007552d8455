export TMPDIR=/tmp
T=${T:-r2w}
mkdir -p gpurun_out/$T
L=dist-svgd_amd/dsvgd/_lib/libdsvgd_hip.so
cp $L /tmp/lib_base.so
AB_VARIANTS='{"x3":{}}' timeout -k 10 300 python scripts/ab_kernels.py --rounds 4 > gpurun_out/$T/ab_base.log 2>&1 && \
cp ${ALT:-ablib_prio.so} $L && \
AB_VARIANTS='{"x3":{}}' timeout -k 10 300 python scripts/ab_kernels.py --rounds 4 > gpurun_out/$T/ab_alt.log 2>&1 && \
cp /tmp/lib_base.so $L && \
AB_VARIANTS='{"x3":{}}' timeout -k 10 300 python scripts/ab_kernels.py --rounds 4 > gpurun_out/$T/ab_base2.log 2>&1
echo rc=$?
for f in ab_base ab_alt ab_base2; do echo $f; grep -A1 '"x3"' gpurun_out/$T/$f.log | grep median; done
