/*
 * JNI binding of libwsgpu (include/wsgpu.h) through libwsgpu_jni (jni/wsgpu_jni.c).
 *
 * The C ABI carries plain pointers and sizes; here every array argument is a
 * direct ByteBuffer (pinned host memory from PinnedByteBufferAllocator when it
 * must cross PCIe at full rate).  Struct layouts (little-endian, see wsgpu.h):
 *   wsg_frame_desc      16 B: u64 payload_off, u32 payload_len, u8 opcode, u8 flags, u16 status
 *   wsg_session_result  16 B: u32 n_delivered, u16 error, u16 close_code, i64 detail
 *   wsg_session_state    8 B
 *   wsg_encode_frame    24 B: u64 payload_off, u32 payload_len, u8 opcode, u8 flags, u8[2], u8[4] mask, u32
 *
 * This repository's image has no JDK: this file is the integration source a
 * maintainer builds (jni/Makefile); the same ABI is exercised from Python
 * (snf4j_amd/_lib.py) by the tests and the bench.
 */
package org.snf4j.websocket.gpu;

import java.nio.ByteBuffer;

final class Wsg {
	/** WSG_BATCHER_MAX_INFLIGHT (wsgpu.h): decode flushes a native batcher keeps in flight. */
	static final int BATCHER_MAX_INFLIGHT = 4;


	static {
		System.loadLibrary("wsgpu_jni");
	}

	private Wsg() {
	}

	/* wsg_status (wsgpu.h), the reference's exception classes */
	static final int OK = 0, E_OPCODE = 1, E_RSV = 2, E_MASKING = 3, E_FRAG_CONTROL = 4, E_CONTROL_LEN = 5,
			E_CLOSE_LEN = 6, E_CONT_OUTSIDE = 7, E_NONCONT_INSIDE = 8, E_MIN_LEN = 9, E_MAX_PAYLOAD = 10,
			E_TOO_LONG = 11, E_CLOSE_STATUS = 12, E_CLOSE_REASON = 13, E_TEXT_UTF8 = 14, E_NEG_LEN = 15,
			E_EXT_LEN = 16, E_BATCH = 17, E_AGG_TOO_BIG = 18, E_INFLATE = 19, E_INFLATE_NO_DATA = 20;

	/** wsg_frame_desc.flags of a batch with stages: an aggregated message (WSG_OUT_AGGREGATED). */
	static final int OUT_AGGREGATED = 0x02;

	static final int DESC_BYTES = 16, RESULT_BYTES = 16, STATE_BYTES = 8, ENCODE_FRAME_BYTES = 24;

	/**
	 * The InvalidFrameException message the reference builds for a status
	 * (FrameDecoder.java:200-255, :390-393; FrameUtf8Validator.java:31).
	 */
	static String message(int status, long detail, long detail2) {
		switch (status) {
		case E_OPCODE: return "Unexpected opcode value (" + detail + ")";
		case E_RSV: return "Unexpected non-zero RSV bits (" + detail + ")";
		case E_MASKING: return "Unexpected payload masking";
		case E_FRAG_CONTROL: return "Fragmented control frame";
		case E_CONTROL_LEN: return "Invalid payload length (" + detail + ") in control frame";
		case E_CLOSE_LEN: return "Invalid payload length (" + detail + ") in close frame";
		case E_CONT_OUTSIDE: return "Continuation frame outside fragmented message";
		case E_NONCONT_INSIDE: return "Non-continuation frame while inside fragmented massage";
		case E_MIN_LEN: return "Invalid minimal payload length";
		case E_MAX_PAYLOAD: return "Invalid maximum payload length";
		case E_TOO_LONG: return "Maximum frame length (" + detail + ") has been exceeded";
		case E_CLOSE_STATUS: return "Invalid close frame status code (" + detail + ")";
		case E_CLOSE_REASON: return "Invalid close frame reason value: bytes are not UTF-8";
		case E_TEXT_UTF8: return "Invalid text frame payload: bytes are not UTF-8";
		case E_NEG_LEN: return "Negative payload length (" + detail + ")";
		case E_EXT_LEN: return "Extended payload length (" + detail + ") > " + detail2;
		case E_AGG_TOO_BIG: return "Too big payload for aggregated frame";
		case E_INFLATE: return "org.snf4j.core.codec.zip.DecompressionException: decompression failure: invalid compressed data format";
		case E_INFLATE_NO_DATA: return "Inflating of input data produced no data";
		default: return "Malformed batch (status " + status + ")";
		}
	}

	/** The CloseFrame status the reference writes for a status (FrameDecoder.java:92-102). */
	static int closeCode(int status) {
		return status == E_CLOSE_REASON || status == E_TEXT_UTF8 ? 1007 : status == E_AGG_TOO_BIG ? 1009 : 1002;
	}

	/* ---- context: wsg_open / wsg_reserve / wsg_close / wsg_last_error ---- */
	static native long open(int device);

	static native int reserve(long ctx, long maxFrames, int maxSessions, long maxWireLen);

	static native void close(long ctx);

	static native String lastError(long ctx);

	/* ---- host framing: FrameDecoder.available (FrameDecoder.java:357-401) ---- */
	/** wsg_frame_available over b[off, off+len); on -1, err = {status, detail, detail2}. */
	static native long frameAvailable(byte[] b, int off, int len, long[] err);

	/** The same over a direct buffer (the IBaseDecoder ByteBuffer overload, :290-332). */
	static native long frameAvailableDirect(ByteBuffer b, int off, int len, long[] err);

	/** wsg_check_header: the header rules of FrameDecoder.decode (:197-256); detail[0] = argument. */
	static native int checkHeader(boolean clientMode, boolean allowExtensions, long maxPayloadLen,
			boolean fragmentation, ByteBuffer data, int off, int len, long[] detail);

	/* ---- cross-session batcher: wsg_batcher_* ---- */
	static native long batcherOpen(long ctx, boolean clientMode, boolean allowExtensions, long maxPayloadLen,
			boolean validateUtf8, int nSessions);

	static native int batcherClose(long batcher);

	/** wsg_batcher_feed: bytes of session sid (copied). */
	static native int batcherFeed(long batcher, int sid, ByteBuffer data, int off, int len);

	static native int batcherFeedArray(long batcher, int sid, byte[] data, int off, int len);

	/**
	 * wsg_batcher_feed_many: one loop iteration's reads in one call.  Read i is session
	 * sids[i]'s bytes [offs[i], offs[i] + lens[i]) of direct[i] (a direct buffer) or, when
	 * that is null, of heap[i]; every read is checked before any is fed.
	 */
	static native int batcherFeedMany(long batcher, int n, int[] sids, ByteBuffer[] direct, byte[][] heap, int[] offs,
			int[] lens);

	/** wsg_batcher_reserve: flushes of up to maxWire bytes / maxFrames frames allocate nothing. */
	static native int batcherReserve(long batcher, long maxWire, long maxFrames);
	static native int batcherReserveStages(long batcher, long maxOutBytes, long maxOutFrames);

	/** wsg_batcher_ticket: the last queued flush's ticket (1, 2, ...). */
	static native long batcherTicket(long batcher);

	/**
	 * wsg_batcher_await (the completion thread, not the loop's): the highest ticket whose
	 * device work has finished, once one above seen has or timeoutMs has passed.
	 */
	static native long batcherAwait(long batcher, long seen, long timeoutMs);

	/**
	 * wsg_batcher_flush: decodes every complete frame fed since the last flush.
	 * views[0..4] receive session_first, desc, payload, result and detail2 wrapped as direct
	 * buffers (valid until the next flush); counts = {n_frames, wire_bytes}.
	 */
	static native int batcherFlush(long batcher, ByteBuffer[] views, long[] counts);

	/** wsg_batcher_flush_async: gather and queue the decode of every complete frame (no wait). */
	static native int batcherFlushAsync(long batcher);

	/** wsg_batcher_wait: the oldest queued flush's results, as batcherFlush gives them. */
	static native int batcherWait(long batcher, ByteBuffer[] views, long[] counts);

	/** wsg_batcher_session_state into st (8 bytes). */
	static native int batcherSessionState(long batcher, int sid, byte[] st);

	/** wsg_batcher_session_reset: slot sid for a new session (a fresh decoder and stages). */
	static native int batcherSessionReset(long batcher, int sid);

	/**
	 * wsg_batcher_set_stages: the decoders after "ws-decoder" each flush runs in the
	 * same device batch (PerMessageDeflateDecoder, FrameUtf8Validator, FrameAggregator).
	 */
	static native int batcherSetStages(long batcher, boolean inflate, boolean noContext, boolean validate,
			boolean aggregate, long maxAggregatedLength);

	/* ---- device per selector loop: wsg_device_for_loop / _account / _release_loop ---- */
	static native int deviceForLoop(long loopId);

	static native int deviceAccount(int device, long wireBytes);

	static native int deviceReleaseLoop(long loopId);

	/* ---- cross-session encode batcher: wsg_enc_batcher_* ---- */
	static native long encBatcherOpen(long ctx, boolean clientMode, int nSessions);

	static native int encBatcherClose(long batcher);

	/** wsg_enc_batcher_add: Frame(opcode, flags = FIN << 7 | RSV << 4, payload) of session sid; mask big-endian. */
	static native int encBatcherAdd(long batcher, int sid, int opcode, int flags, int mask, byte[] payload);

	/** wsg_enc_batcher_flush: views = {session_first, wire_off, wire} (valid until the next add / flush). */
	static native int encBatcherFlush(long batcher, ByteBuffer[] views);

	/** wsg_enc_batcher_flush_async: queue the encode of everything added so far (at most two in flight). */
	static native int encBatcherFlushAsync(long batcher);

	/** wsg_enc_batcher_wait: the oldest in-flight flush's views (null: discard them). */
	static native int encBatcherWait(long batcher, ByteBuffer[] views);

	static native int encBatcherSessionReset(long batcher, int sid);

	static native int encBatcherReserve(long batcher, long maxFrames, long maxPayload);

	/** wsg_enc_batcher_set_deflate: PerMessageDeflateEncoder(level, noContext) in front of the encoder, on the device. */
	static native int encBatcherSetDeflate(long batcher, int level, boolean noContext);

	static native long encBatcherTicket(long batcher);

	static native long encBatcherAwait(long batcher, long seen, long timeoutMs);

	/* ---- encode: wsg_encoded_length / wsg_encode_batch_host ---- */
	static native long encodedLength(int payloadLen, boolean clientMode);

	static native int encodeBatchHost(long ctx, boolean clientMode, ByteBuffer payload, long payloadLen,
			ByteBuffer frames, long nFrames, ByteBuffer sessionFirst, int nSessions, ByteBuffer closed,
			ByteBuffer wireOut, long wireCap, ByteBuffer wireOff);

	/* ---- validator stage alone: wsg_validate_batch_host ---- */
	static native int validateBatchHost(long ctx, ByteBuffer desc, long nFrames, ByteBuffer sessionFirst,
			int nSessions, ByteBuffer payload, long payloadLen, ByteBuffer state, ByteBuffer result);

	/* ---- opening handshake: wsg_handshake_available / wsg_handshake_accept_batch_host /
	 * wsg_handshake_validate_batch_host (the GpuHandshakeDecoder stages of INTEGRATION.md
	 * 1.3d-e).  config = {maxLength, ignoreHost, subprotocols, extensions, hostPolicy}
	 * as wsg_hs_config; results are 16-byte wsg_hs_result records. ---- */
	static native int handshakeAvailable(byte[] b, int off, int len);

	static native int handshakeAcceptBatchHost(long ctx, int[] config, ByteBuffer req, ByteBuffer reqOff, int n,
			ByteBuffer resp, ByteBuffer result);

	static native int handshakeValidateBatchHost(long ctx, int[] config, ByteBuffer resp, ByteBuffer respOff,
			ByteBuffer keys, int n, ByteBuffer expected, ByteBuffer result);

	/* ---- pinned host pool: wsg_host_alloc / wsg_host_release ---- */
	static native ByteBuffer allocPinned(int capacity);

	static native int releasePinned(ByteBuffer buffer);
}
