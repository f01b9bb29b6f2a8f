export TMPDIR=/tmp
CONFIGS="n256" bash tools/pmc_configs.sh r03aj
