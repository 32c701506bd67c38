"""Lifecycle state machines (reference polyaxon/constants/*)."""
from polyaxon_amd.fsm.lifecycles import (S, BuildJobLifeCycle, ExperimentGroupLifeCycle,  # noqa: F401
                                         ExperimentLifeCycle, JobLifeCycle, Lifecycle, OperationLifeCycle,
                                         PipelineLifeCycle, PluginLifeCycle, TriggerPolicy)
