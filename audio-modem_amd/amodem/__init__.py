"""amodem — MI355X-native OFDM demodulator (host mirror of modem.js over libamodem)."""
from . import _lib
from .modem import (STREAM_FRAME_DTYPE, AssemblerError, ChunkAssembler, StreamingReceiver, DeviceGroup, ResidentBatch, Pipeline, FRAME_DATA, FRAME_META, OFDM, OFDM_CONFIGS, RESULT_DTYPE, Demodulator, build_data_chunk_frame,
                    build_metadata_frame, build_transmit_signal, crc32, estimate_frame_samples,
                    generate_preamble_symbol1, generate_test_signal, make_cfg, num_data_subs, packet_chunk, packet_legacy,
                    packet_meta, payload_stride, preset, set_ofdm_config, synth_legacy_batch, synth_legacy_packets,
                    synth_payload, to_reference, tx_silence)

__all__ = ["Demodulator", "ChunkAssembler", "StreamingReceiver", "DeviceGroup", "ResidentBatch", "Pipeline", "AssemblerError", "OFDM", "OFDM_CONFIGS", "FRAME_META", "FRAME_DATA", "RESULT_DTYPE", "set_ofdm_config",
           "make_cfg", "preset", "crc32", "payload_stride", "estimate_frame_samples", "generate_preamble_symbol1",
           "build_transmit_signal", "build_metadata_frame", "build_data_chunk_frame", "generate_test_signal",
           "synth_payload", "synth_legacy_batch", "to_reference", "packet_legacy", "packet_meta", "packet_chunk",
           "tx_silence", "synth_legacy_packets", "num_data_subs"]
