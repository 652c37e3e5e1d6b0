from .misc import (AverageMeter, ProgressBar, accuracy, accuracy_from_rank, check_folder, check_integrity,
                   download_url, format_time, list_dir, list_files, makedir_exist_ok, progress_bar, rank0_print,
                   set_seed, worker_init_fn)

__all__ = ["AverageMeter", "ProgressBar", "accuracy", "accuracy_from_rank", "check_folder", "check_integrity",
           "download_url", "format_time", "list_dir", "list_files", "makedir_exist_ok", "progress_bar",
           "rank0_print", "set_seed", "worker_init_fn"]
