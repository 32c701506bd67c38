"""Polyaxonfile specification layer (replaces the reference's external ``polyaxon_schemas``)."""
from polyaxon_amd.spec.hptuning import HPTuningConfig, Optimization, SearchAlgorithms  # noqa: F401
from polyaxon_amd.spec.matrix import MatrixConfig, MatrixValidationError  # noqa: F401
from polyaxon_amd.spec.specification import (BuildSpecification, ExperimentSpecification,  # noqa: F401
                                             GroupSpecification, JobSpecification, Kinds, NotebookSpecification,
                                             PipelineSpecification, PolyaxonfileError, TensorboardSpecification,
                                             specification_for, validate)
from polyaxon_amd.spec.specification import read_raw as read_raw_spec  # noqa: F401,E402
