bash tools/pmc_configs.sh r04u
