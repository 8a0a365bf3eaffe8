"""REDCLIFF_S_CMLP (models/redcliff_s_cmlp.py) on MI355X: the base class without the
factor-weight smoothing penalty.  compute_loss returns the reference's 6-term list and
validate_training its 9-value tuple.  The reference's GPU-only crash at
models/redcliff_s_cmlp.py:360-361 (undefined ``in_x``) is deliberately not reproduced."""
from .redcliff_s_cmlp_withStateSmoothing import REDCLIFF_S_CMLP_withStateSmoothing


class REDCLIFF_S_CMLP(REDCLIFF_S_CMLP_withStateSmoothing):
    _WITH_SMOOTHING = False

    def __init__(self, num_chans, gen_lag, gen_hidden, embed_lag, embed_hidden_sizes, num_in_timesteps,
                 num_out_timesteps, num_factors, num_supervised_factors, coeff_dict, use_sigmoid_restriction,
                 factor_score_embedder_type, factor_score_embedder_args, primary_gc_est_mode, forward_pass_mode,
                 num_sims=1, wavelet_level=None, save_path=None,
                 training_mode="pretrain_embedder_and_pretrain_factor_then_combined", num_pretrain_epochs=0,
                 num_acclimation_epochs=0):
        super().__init__(num_chans, gen_lag, gen_hidden, embed_lag, embed_hidden_sizes, num_in_timesteps,
                         num_out_timesteps, num_factors, num_supervised_factors, coeff_dict, use_sigmoid_restriction,
                         factor_score_embedder_type, factor_score_embedder_args, primary_gc_est_mode,
                         forward_pass_mode, num_sims=num_sims, wavelet_level=wavelet_level, save_path=save_path,
                         training_mode=training_mode, num_pretrain_epochs=num_pretrain_epochs,
                         num_acclimation_epochs=num_acclimation_epochs)
