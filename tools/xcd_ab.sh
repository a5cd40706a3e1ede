set -o pipefail
PMC_LIBS="x16: x32:var/libx32.so x64:var/libx64.so x128:var/libx128.so x4:var/libx4.so" PMC="FETCH_SIZE" PMC_ARGS="--config 4 --opt modes_overlap=0" bash tools/pmc_ab.sh gpurun_out/xcd "k_boot_gene" > gpurun_out/xcd.txt 2>&1 || exit 1
KT_LIBS="x16: x32:var/libx32.so x64:var/libx64.so x128:var/libx128.so x4:var/libx4.so" KT_ARGS="--config 4 --opt modes_overlap=0" bash tools/ktrace_ab.sh gpurun_out/xcdk "k_boot_gene" >> gpurun_out/xcd.txt 2>&1 || exit 1
KT_LIBS="x16: x32:var/libx32.so x64:var/libx64.so x128:var/libx128.so" KT_ARGS="--config 3 --opt lanes=1" bash tools/ktrace_ab.sh gpurun_out/xcdk3 "k_boot_gene" >> gpurun_out/xcd.txt 2>&1
