"""Reference players/player_alpha.py surface: 5000 simulations, no noise."""
from players._alpha_base import AlphaPlayer


class Player(AlphaPlayer):
    def __init__(self, rules="gomoku", board_size=15, n_simulations=5000, c_puct=1.0,
                 model_path="models/snapshot_iter140_20260109_190822.pt", nn_model=None,
                 mcts_class=None):
        super().__init__(rules, board_size, n_simulations, c_puct, model_path, nn_model,
                         mcts_class=mcts_class)
