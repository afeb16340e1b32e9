# round-6 profiles of the final tree: graph/eager kernel stats, FETCH/WRITE PMC passes, 3bp/mnist graph stats
bash tools/refresh_profiles.sh r06 || exit 1
bash tools/prof_configs.sh r06 || exit 1
