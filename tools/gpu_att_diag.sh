set -o pipefail
timeout -k 10 120 python -u tools/att_prod_bf16_diag.py && ASR_LSTM_XG=0 timeout -k 10 120 python -u tools/att_prod_bf16_diag.py && ASR_LSTM_PERSIST=0 timeout -k 10 120 python -u tools/att_prod_bf16_diag.py
