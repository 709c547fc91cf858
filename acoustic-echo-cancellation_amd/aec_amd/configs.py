"""Configuration dicts the hot path reads — same keys and values as the
reference's scripts/configs.py:1-46 (speech_conf, train_conf, erb_conf, net_conf)."""

speech_conf = {
    'in_norm': True,
    'sample_rate': 16000,
    'win_len': 0.032,
    'hop_len': 0.016,
    'win_size': 512,
    'hop_size': 256,
}

train_conf = {
    'logging_period': 1,
    'lr': 0.00001,
    'lr_decay_factor': 0.5,
    'lr_decay_period': 5,
    'clip_norm': -1,
    'max_n_epochs': 50,
    'batch_size': 16,
    'gpu_ids': [0],
}

erb_conf = {
    'nfreqs': 257,
    'sample_rate': 16000,
    'total_erb_bands': 32,
    'low_freq': 0,
    'max_freq': 8000,
}

# DCCRN config (scripts/configs.py:29-46), read by dccrn.DCCRN / dccrn2.DCCRN
net_conf = {
    'win_size': 512,
    'hop_size': 256,
    'samplerates': 16000,
    'win_type': 'hann',
    'hidden_dim': 4,
    'rnn_layers': 2,
    'rnn_units': 128,
    'use_clstm': True,
    'use_cbn': True,
    'masking_mode': 'E',
    'conv_channels': [4, 16, 32, 64, 128, 256, 512],
    'kernel_size': (5, 1),
    'stride': (2, 1),
    'padding': (2, 0),
    'dilation': 1,
    'groups': 1,
}

# Build-defined FD-NLMS defaults (no reference counterpart).
nlms_conf = {
    'taps': 4,
    'mu': 0.3,
    'beta': 0.5,
    'delta': 1e-4,
}
