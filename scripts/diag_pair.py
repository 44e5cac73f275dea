from distributed_char_rnn_amd.ops import native
o = native.ops()
for H, B in [(128, 32), (512, 256), (384, 64), (256, 96)]:
    print(H, B, "fwd2", o.lstm2_persist_supported(H, B), "bwd2", o.lstm2_bwd_persist_supported(H, B))
