from .train_flows import DataParallel, get_params, nll_step, set_params, train

__all__ = ["DataParallel", "get_params", "nll_step", "set_params", "train"]
