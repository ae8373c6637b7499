"""fleet.data_generator (reference: python/paddle/distributed/fleet/data_generator/data_generator.py):
user-defined line parsers that emit the MultiSlot text format read by the parameter-server data
feeds.  A sample is a list of (slot_name, values); each slot is written as "<len> v1 v2 ..." and
the slots of one sample are space-joined on one line."""
import sys


class DataGenerator:
    def __init__(self):
        self._proto_info = None
        self.batch_size_ = 32

    def set_batch(self, batch_size):
        self.batch_size_ = batch_size

    def generate_sample(self, line):
        """Override: return a callable yielding samples [(name, values), ...] for one input line."""
        raise NotImplementedError("implement generate_sample(line) in the DataGenerator subclass")

    def generate_batch(self, samples):
        """Override for batch-level processing (e.g. padding); default passes samples through."""
        def local_iter():
            for s in samples:
                yield s
        return local_iter

    def _emit(self, batch, out):
        for s in self.generate_batch(batch)():
            out.write(self._gen_str(s))

    def _run(self, lines, out):
        batch = []
        for line in lines:
            for sample in self.generate_sample(line)():
                if sample is None:
                    continue
                batch.append(sample)
                if len(batch) == self.batch_size_:
                    self._emit(batch, out)
                    batch = []
        if batch:
            self._emit(batch, out)

    def run_from_stdin(self):
        self._run(sys.stdin, sys.stdout)

    def run_from_memory(self):
        """Generates from generate_sample(None) (debugging / benchmarking)."""
        self._run([None], sys.stdout)

    def _gen_str(self, line):
        raise NotImplementedError

    @staticmethod
    def _check(line):
        if isinstance(line, zip):
            line = list(line)
        if not isinstance(line, (list, tuple)):
            raise ValueError("a sample must be a list/tuple of (slot_name, values), "
                             "e.g. [('words', [1926, 8, 17]), ('label', [1])]")
        return line


class MultiSlotStringDataGenerator(DataGenerator):
    def _gen_str(self, line):
        parts = []
        for name, elements in self._check(line):
            parts.append(" ".join([str(len(elements))] + [str(e) for e in elements]))
        return " ".join(parts) + "\n"


class MultiSlotDataGenerator(DataGenerator):
    """Numeric slots; the first sample fixes the slot names and types (uint64 unless a float
    appears, which turns the slot to float for the rest of the stream)."""

    def _gen_str(self, line):
        line = self._check(line)
        if self._proto_info is None:
            self._proto_info = []
            for name, elements in line:
                if not isinstance(name, str):
                    raise ValueError(f"slot name must be str, got {type(name)}")
                if not isinstance(elements, list) or not elements:
                    raise ValueError(f"slot {name}: values must be a non-empty list (pad in generate_sample)")
                self._proto_info.append((name, "uint64"))
        elif len(line) != len(self._proto_info):
            raise ValueError("every sample must carry the same slots as the first one")
        parts = []
        for i, (name, elements) in enumerate(line):
            if name != self._proto_info[i][0]:
                raise ValueError(f"slot {i} is {name}, expected {self._proto_info[i][0]}")
            if not isinstance(elements, list) or not elements:
                raise ValueError(f"slot {name}: values must be a non-empty list")
            for e in elements:
                if isinstance(e, float):
                    self._proto_info[i] = (name, "float")
                elif not isinstance(e, int):
                    raise ValueError(f"slot {name}: values must be int or float, got {type(e)}")
            parts.append(" ".join([str(len(elements))] + [str(e) for e in elements]))
        return " ".join(parts) + "\n"
