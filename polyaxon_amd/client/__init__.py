"""Tracking client and in-cluster helpers (reference polyaxon-client / polyaxon-helper)."""
from polyaxon_amd.client.tracking import (Experiment, MetricStream, get_cluster_def, get_data_paths,  # noqa: F401
                                          get_declarations, get_experiment_info, get_job_info, get_log_level,
                                          get_outputs_path, get_outputs_refs_paths, get_task_index, get_task_info,
                                          get_task_type, get_tf_config, is_in_cluster)
