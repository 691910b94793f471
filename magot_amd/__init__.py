"""magot_amd -- MI355X-native drop-in for MAGOT's CDS extraction path.

``from magot_amd import genome`` gives the reference's ``genome`` module API
(Genome, GenomeSequence, AnnotationSet, BaseAnnotation, ParentAnnotation,
Sequence, read_gff, ensure_file); sequence work runs in libmagot.so on the GPU.
"""

from . import genome  # noqa: F401
from .genome import (AnnotationSet, BaseAnnotation, Genome, GenomeSequence,  # noqa: F401
                     ParentAnnotation, Sequence, ensure_file, read_gff)

__version__ = '0.1.0'
