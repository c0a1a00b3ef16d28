/*
 * The "ws-encoder" stage: FrameEncoder (FrameEncoder.java:41-136) with the header
 * emit and the client-side masking of large frames on the MI355X
 * (wsg_encode_batch_host, k_enc_* kernels).  Small frames are header bytes plus a
 * short copy, cheaper on the loop thread than a PCIe round trip: they go through
 * the reference's own FrameEncoder.  The mask comes from the same
 * java.util.Random stream as FrameEncoder.RANDOM (:43,111); the close latch
 * (:71-76) is the `closed` byte passed to the device.  Output buffers come from
 * session.allocate (:78) and belong to the session writer.
 */
package org.snf4j.websocket.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.List;
import java.util.Random;

import org.snf4j.core.codec.IEncoder;
import org.snf4j.core.session.ISession;
import org.snf4j.websocket.frame.Frame;
import org.snf4j.websocket.frame.FrameEncoder;
import org.snf4j.websocket.frame.Opcode;

public class GpuFrameEncoder implements IEncoder<Frame, ByteBuffer> {

	private static final Random RANDOM = new Random();
	/** frames with at least this many payload bytes are encoded on the device */
	private final int deviceThreshold;
	private final boolean clientMode;
	private final FrameEncoder small;
	private final WsgBatcher batcher;
	private final ByteBuffer closed = ByteBuffer.allocateDirect(1);
	private final ByteBuffer sessionFirst = ByteBuffer.allocateDirect(8).order(ByteOrder.LITTLE_ENDIAN);
	private final ByteBuffer frameRec = ByteBuffer.allocateDirect(Wsg.ENCODE_FRAME_BYTES).order(ByteOrder.LITTLE_ENDIAN);
	private final ByteBuffer wireOff = ByteBuffer.allocateDirect(16).order(ByteOrder.LITTLE_ENDIAN);

	public GpuFrameEncoder(boolean clientMode, WsgBatcher batcher, int deviceThreshold) {
		this.clientMode = clientMode;
		this.batcher = batcher;
		this.deviceThreshold = deviceThreshold;
		this.small = new FrameEncoder(clientMode);
		sessionFirst.putInt(0, 0).putInt(4, 1);
	}

	@Override
	public Class<Frame> getInboundType() {
		return Frame.class;
	}

	@Override
	public Class<ByteBuffer> getOutboundType() {
		return ByteBuffer.class;
	}

	@Override
	public void encode(ISession session, Frame frame, List<ByteBuffer> out) throws Exception {
		if (closed.get(0) != 0)
			return;  // FrameEncoder.java:71-76
		if (frame.getPayloadLength() < deviceThreshold) {
			small.encode(session, frame, out);
			if (frame.getOpcode() == Opcode.CLOSE)
				closed.put(0, (byte) 1);
			return;
		}
		byte[] p = frame.getPayload();
		ByteBuffer payload = session.allocate(p.length);
		payload.put(p).flip();
		int len = (int) Wsg.encodedLength(p.length, clientMode);
		ByteBuffer wire = session.allocate(len);
		frameRec.clear();
		frameRec.putLong(0, 0).putInt(8, p.length).put(12, (byte) frame.getOpcode().value())
				.put(13, (byte) ((frame.isFinalFragment() ? 0x80 : 0) | (frame.getRsvBits() << 4)));
		if (clientMode) {
			byte[] mask = new byte[4];
			RANDOM.nextBytes(mask);
			for (int i = 0; i < 4; ++i)
				frameRec.put(16 + i, mask[i]);
		}
		int rc = Wsg.encodeBatchHost(batcher.ctx, clientMode, direct(payload), p.length, frameRec, 1, sessionFirst, 1,
				closed, direct(wire), len, wireOff);
		session.release(payload);
		if (rc != 0)
			throw new IllegalStateException("wsg_encode_batch_host: " + Wsg.lastError(batcher.ctx));
		wire.position(0).limit(len);
		out.add(wire);
	}

	/** Session buffers must be direct to cross JNI (PinnedByteBufferAllocator gives pinned ones). */
	private static ByteBuffer direct(ByteBuffer b) {
		if (!b.isDirect())
			throw new IllegalStateException("GpuFrameEncoder needs a direct-buffer allocator");
		return b;
	}
}
