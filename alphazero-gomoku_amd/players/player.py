"""Reference players/player.py (== player_alpha2.py) surface: 3000 simulations, noise params set but off."""
from players._alpha_base import AlphaPlayer


class Player(AlphaPlayer):
    def __init__(self, rules="gomoku", board_size=15, n_simulations=3000, c_puct=1.0,
                 model_path="models/snapshot_iter83_20251207_091724.pt", nn_model=None,
                 mcts_class=None):
        super().__init__(rules, board_size, n_simulations, c_puct, model_path, nn_model,
                         mcts_kwargs=dict(dirichlet_alpha=0.03, epsilon=0.03, apply_dirichlet_n_first_moves=10), mcts_class=mcts_class)
