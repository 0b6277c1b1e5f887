set -o pipefail
timeout -k 5 60 tools/ubench/fold_lds
